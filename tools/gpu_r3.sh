# Round-3 GPU pass: gpu tests, smoke, the default bench line, and a rocprofv3 kernel trace of the
# headline workload alone (reconciled with its own bench line by tools/trace_steps.py).
# usage: bash tools/gpu_r2.sh TAG
set -o pipefail
T=${1:-r3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err &&
bash tools/gpu_prof.sh ${T}
