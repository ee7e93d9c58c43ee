# Round-4 pass E: the screened-argmax split per input kind, the GPU suite, the dev build's STFT /
# subtract parity, an interleaved A/B (this build, the dev build, the two selection-sort variants),
# the subtract leg on both builds, and the bench line.   usage: bash tools/gpu_r4e.sh TAG
# A step that fails its tests does not stop the pass; a time limit, abort or crash (rc >= 124) does.
set -o pipefail
T=${1:-r4e}
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
PYT="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
run screen 300 $PYT -s tests/test_gpu_drift.py -k screened
run tests 900 $PYT -x tests
FT8HIP_LIB=$R/variants/DEV.so FT8HIP_ALLOW_STALE=1 run devtests 600 $PYT -x tests/test_gpu_stft.py tests/test_gpu_e2e.py tests/test_gpu_tx.py tests/test_gpu_bench_parity.py tests/test_gpu_subtract_oracle.py
run ab 900 python -u tools/ab_variants.py $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/DEV.so $R/variants/BITONIC.so $R/variants/RANK.so
for i in 1 2; do
  FT8HIP_LIB=$R/ft8_demodulator_amd/lib/libft8hip.so FT8HIP_ALLOW_STALE=1 run sub_main$i 300 python -u tools/experiments/sub_bench.py
  FT8HIP_LIB=$R/variants/DEV.so FT8HIP_ALLOW_STALE=1 run sub_dev$i 300 python -u tools/experiments/sub_bench.py
done
run bench 600 python -u bench.py
