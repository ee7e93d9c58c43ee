# Round-4 pass F: a dev build against this one -- the second pass's residual / fit digests on both
# (bit-identity), the dev build's subtract and end-to-end tests, and the subtract leg interleaved.
#   usage: bash tools/gpu_r4f.sh TAG    (variants/DEV.so = the dev build)
set -o pipefail
T=${1:-r4f}
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
MAIN=$R/ft8_demodulator_amd/lib/libft8hip.so
DEV=$R/variants/DEV.so
PYT="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
FT8HIP_LIB=$MAIN FT8HIP_ALLOW_STALE=1 run digest_main 300 python -u tools/experiments/sub_digest.py
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run digest_dev 300 python -u tools/experiments/sub_digest.py
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run devtests 600 $PYT -x tests/test_gpu_tx.py tests/test_gpu_subtract_oracle.py tests/test_gpu_e2e.py tests/test_gpu_stft.py tests/test_gpu_stages.py tests/test_gpu_bench_parity.py tests/test_gpu_reftests.py
run ab 900 python -u tools/ab_variants.py $MAIN $DEV
for i in 1 2; do
  FT8HIP_LIB=$MAIN FT8HIP_ALLOW_STALE=1 run sub_main$i 300 python -u tools/experiments/sub_bench.py
  FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run sub_dev$i 300 python -u tools/experiments/sub_bench.py
done
