# A/B of library variants (variants/*.so): BP/stage parity tests on each candidate variant, then
# interleaved timing rounds (tools/ab_variants.py).  usage: TESTED="A B" bash tools/gpu_ab.sh TAG O A B
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
for v in ${TESTED:-}; do
  FT8HIP_LIB=$PWD/variants/$v.so FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_e2e.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${T}_t_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u tools/ab_variants.py $(for v in "$@"; do echo $PWD/variants/$v.so; done) > gpurun_out/${T}_ab.log 2>&1
