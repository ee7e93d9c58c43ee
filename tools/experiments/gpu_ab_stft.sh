# STFT A/B: STFT + e2e parity tests on the candidate variants, then interleaved timing rounds.
# usage: TESTED="P" bash tools/experiments/gpu_ab_stft.sh TAG O P
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
for v in ${TESTED:-}; do
  FT8HIP_LIB=$PWD/variants/$v.so FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_stft.py tests/test_gpu_e2e.py tests/test_gpu_reftests.py tests/test_gpu_bench_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/${T}_t_$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u tools/ab_variants.py $(for v in "$@"; do echo $PWD/variants/$v.so; done) > gpurun_out/${T}_ab.log 2>&1
