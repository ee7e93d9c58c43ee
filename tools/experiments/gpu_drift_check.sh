set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_drift.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/d1.log 2>&1
rc=$?
if [ $rc -eq 0 ]; then timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/d1all.log 2>&1; fi
