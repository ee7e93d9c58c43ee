# Round-4 pass I: the STFT tests (the int16 == float32 case of the packed plans), on this build and
# on variants/PK2.so (k_stft_pk's full-band pair epilogue); the geometry legs, this build against
# PK2; an interleaved A/B of k_stft3840p run lengths (variants/CH4.so, CH8.so, CH12.so against 6).
#   usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
T=${1:-r4i}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  local name=$1 to=$2
  shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/${T}_steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
PYT="python -u -m pytest -v -rP --timeout 120 --timeout-method thread -m gpu"
run stft_tests 300 $PYT tests/test_gpu_stft.py
FT8HIP_LIB=$R/variants/PK2.so FT8HIP_ALLOW_STALE=1 run pk2_tests 300 $PYT tests/test_gpu_stft.py tests/test_gpu_reftests.py
for i in 1 2; do
  FT8HIP_LIB=$R/ft8_demodulator_amd/lib/libft8hip.so FT8HIP_ALLOW_STALE=1 run geo_main$i 300 python -u tools/experiments/geo_bench.py
  FT8HIP_LIB=$R/variants/PK2.so FT8HIP_ALLOW_STALE=1 run geo_pk2$i 300 python -u tools/experiments/geo_bench.py
done
run chunk_ab 800 python -u tools/ab_variants.py $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/CH4.so $R/variants/CH8.so $R/variants/CH12.so
