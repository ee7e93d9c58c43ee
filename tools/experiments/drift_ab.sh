# A/B of the drift-correction leg for alternative library builds (variants/*.so via FT8HIP_LIB)
set -o pipefail
mkdir -p gpurun_out
FT8HIP_LIB=$PWD/variants/O.so timeout -k 10 200 python -u tools/experiments/drift_bench.py 64 > gpurun_out/dab_warm.log 2>&1 || exit 1
for v in ${VARIANTS:-O A B}; do
  FT8HIP_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u tools/experiments/drift_bench.py > gpurun_out/dab_$v.log 2> gpurun_out/dab_$v.err || exit 1
done
for v in ${TESTED:-A B}; do
  FT8HIP_LIB=$PWD/variants/$v.so timeout -k 10 200 python -u -m pytest tests/test_gpu_drift.py tests/test_gpu_stft.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/dab_t_$v.log 2>&1 || exit 1
done
