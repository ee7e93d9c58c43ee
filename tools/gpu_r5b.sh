# Round-5 pass B: the GPU suite on the current tree, then same-box interleaved A/B of the round-4
# library (variants/R4.so, tools/build_ref_variant.sh R4 7a59f02) against this build: the
# subtract-and-redecode leg, the geometry legs and the headline step (tools/ab_variants.py).
set -o pipefail
T=${1:-r5b}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
for r in 1 2; do
  for L in R4 HEAD; do
    if [ $L = R4 ]; then LIB=$R/variants/R4.so; else LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; fi
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/${T}_sub_${L}_$r.log 2>&1 || exit 1
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py > gpurun_out/${T}_geo_${L}_$r.log 2>&1 || exit 1
  done
done &&
timeout -k 10 600 python -u tools/ab_variants.py $R/variants/R4.so $R/ft8_demodulator_amd/lib/libft8hip.so > gpurun_out/${T}_ab.log 2>&1
