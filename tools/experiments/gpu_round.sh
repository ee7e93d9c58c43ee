# One full round on the GPU box: gpu tests, smoke, the default bench line, and the rocprofv3
# kernel statistics of the headline workload and of the drift leg (tools/experiments/gpu_profiles.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/t12.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s12.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/b12.log 2> gpurun_out/b12.err &&
bash tools/experiments/gpu_profiles.sh
