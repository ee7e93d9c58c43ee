# Round-5 pass D: GPU suite; same-box A/B of the headline step (round-4 library, this build, and
# variant W = k_stft3840p with the window read from L1 instead of LDS); the subtract leg (round-4 vs
# this build); then the full bench line.
set -o pipefail
T=${1:-r5d}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_variants.py $R/variants/R4.so $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/W.so > gpurun_out/${T}_ab.log 2>&1 &&
for r in 1 2; do
  for L in R4 HEAD; do
    if [ $L = R4 ]; then LIB=$R/variants/R4.so; else LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; fi
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/${T}_sub_${L}_$r.log 2>&1 || exit 1
  done
done &&
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err
