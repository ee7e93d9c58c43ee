# Round-4 pass D: GPU tests, an interleaved A/B of the selection sorts (LDS bitonic, rank sort,
# this build's register network), and the bench line.   usage: bash tools/gpu_r4d.sh TAG
set -o pipefail
T=${1:-r4d}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_variants.py $R/variants/BITONIC.so $R/variants/RANK.so $R/ft8_demodulator_amd/lib/libft8hip.so > gpurun_out/${T}_sortab.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err
