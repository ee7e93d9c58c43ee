# Round-4 pass A: GPU tests on the in-tree build, an interleaved k_bp A/B (round-2 bp.hip, round-3
# HEAD, this build), then the GPU tests once more on the barrier-race check build (variants/RACE.so,
# tools/build_race.sh).   usage: bash tools/gpu_r4a.sh TAG
set -o pipefail
T=${1:-r4a}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_variants.py $R/variants/R2BP.so $R/variants/R3HEAD.so $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/R2BP.so $R/variants/R3HEAD.so $R/ft8_demodulator_amd/lib/libft8hip.so > gpurun_out/${T}_bpab.log 2>&1 &&
FT8HIP_LIB=$R/variants/RACE.so FT8HIP_ALLOW_STALE=1 timeout -k 10 900 python -u -m pytest tests -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_race_tests.log 2>&1
