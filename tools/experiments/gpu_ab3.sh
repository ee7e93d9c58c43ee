# Round-3 kernel change pass: gpu tests, an interleaved A/B of a variant library against the
# in-tree build (tools/ab_variants.py), then a kernel trace of the headline workload.
# usage: bash tools/gpu_ab3.sh TAG variants/OLD.so
set -o pipefail
T=${1:-r3ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_variants.py $2 $GRAFT_REPO_ROOT/ft8_demodulator_amd/lib/libft8hip.so > gpurun_out/${T}_ab.log 2>&1 &&
bash tools/gpu_prof.sh ${T}
