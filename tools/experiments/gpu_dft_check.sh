set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_stft.py tests/test_gpu_drift.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/dft.log 2>&1
