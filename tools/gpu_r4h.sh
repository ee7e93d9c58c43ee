# Round-4 pass H: the bench line and the headline kernel trace again on another box (box clocks
# differ: the same build's kernels take the same cycles at different frequencies).
#   usage: bash tools/gpu_r4h.sh TAG
set -o pipefail
T=${1:-r4h}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err &&
bash tools/gpu_prof.sh ${T}
