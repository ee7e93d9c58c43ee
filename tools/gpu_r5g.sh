# chirp-z 512-thread variant: STFT/drift/harness tests on the current build, then interleaved A/B of
# the 32 768 Hz drift leg against variants/O.so (the committed csrc)
set -o pipefail
mkdir -p gpurun_out
T="${1:-r5g}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_stft.py tests/test_gpu_drift.py tests/test_gpu_harness.py -x -q \
  --timeout 120 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  FT8HIP_LIB=$PWD/variants/O.so FT8HIP_ALLOW_STALE=1 timeout -k 10 200 python -u tools/experiments/drift32_bench.py \
    >> gpurun_out/${T}_ab_O.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/experiments/drift32_bench.py >> gpurun_out/${T}_ab_N.log 2>&1 || exit 1
done
