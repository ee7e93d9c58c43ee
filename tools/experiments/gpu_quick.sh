# quick check: GPU tests of the touched stage + the headline bench without side legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/q_t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress > gpurun_out/q_b.log 2> gpurun_out/q_b.err
