set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_tx.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/sub_t.log 2>&1 &&
timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/sub_b.log 2>&1
