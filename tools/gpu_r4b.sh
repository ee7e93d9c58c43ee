# Round-4 pass B: GPU tests, the bench line, the subtract-leg profile (tools/gpu_sub_prof.sh).
#   usage: bash tools/gpu_r4b.sh TAG
set -o pipefail
T=${1:-r4b}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err &&
bash tools/gpu_sub_prof.sh ${T}
