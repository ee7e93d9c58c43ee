# Round-4 pass C: GPU tests, the bench line, the subtract-leg profile, and the N > 1 rehearsal
# (two ranks on cuda:0 over gloo: per-rank oracle samples vs the gathered decodes).
#   usage: bash tools/gpu_r4c.sh TAG
set -o pipefail
T=${1:-r4c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err &&
bash tools/gpu_sub_prof.sh ${T} &&
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 > gpurun_out/${T}_rehearse2.log 2> gpurun_out/${T}_rehearse2.err
