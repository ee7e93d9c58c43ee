# Round-3 quick pass: gpu tests, then a kernel trace of the headline workload (no CPU / side legs).
# usage: bash tools/gpu_quick3.sh TAG
set -o pipefail
T=${1:-r3q}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
bash tools/gpu_prof.sh ${T}
