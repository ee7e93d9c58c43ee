# Round-5 pass E: GPU suite, the subtract leg (this build, twice), the headline kernel trace
# (tools/gpu_prof.sh) and the subtract leg's trace + counter passes (tools/gpu_sub_prof.sh).
set -o pipefail
T=${1:-r5e}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/${T}_sub_1.log 2>&1 &&
timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/${T}_sub_2.log 2>&1 &&
bash tools/gpu_prof.sh ${T} &&
bash tools/gpu_sub_prof.sh ${T}
# then pass F's score-kernel variants (tools/gpu_r5f.sh)
[ $? -eq 0 ] && bash tools/gpu_r5f.sh r5f
