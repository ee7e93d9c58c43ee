# A/B: headline bench stage times for alternative library builds (variants/*.so via FT8HIP_LIB),
# then the GPU parity tests of the stages and the end-to-end path on each variant
set -o pipefail
mkdir -p gpurun_out
# a throwaway first run: the first bench of a call on a fresh box runs a few % slow
FT8HIP_LIB=$PWD/variants/O.so timeout -k 10 200 python -u bench.py --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress --steps 5 > gpurun_out/ab_warm.log 2>&1 || exit 1
for v in ${VARIANTS:-O A B}; do
  FT8HIP_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress > gpurun_out/ab_$v.log 2> gpurun_out/ab_$v.err || exit 1
done
for v in ${TESTED:-A B}; do
  FT8HIP_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stages.py tests/test_gpu_e2e.py tests/test_gpu_stft.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/ab_t_$v.log 2>&1 || exit 1
done
