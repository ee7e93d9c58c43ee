# Round-5 pass F: k_score2 with difference tiles (variants DV: 78 VGPRs, DV8: 64 VGPRs under an
# 8-waves-per-SIMD budget) -- their score grids against the goldens / oracle (the stage tests on the
# variant library), then a same-box interleaved A/B of the headline step against this build.
set -o pipefail
T=${1:-r5f}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
for V in DV DV8; do
  FT8HIP_LIB=$R/variants/$V.so FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stages.py tests/test_gpu_reftests.py tests/test_gpu_bench_parity.py > gpurun_out/${T}_tests_$V.log 2>&1 || exit 1
done &&
timeout -k 10 600 python -u tools/ab_variants.py $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/DV.so $R/variants/DV8.so > gpurun_out/${T}_ab.log 2>&1 &&
for V in HEAD DV; do
  if [ $V = HEAD ]; then LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; else LIB=$R/variants/$V.so; fi
  FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py > gpurun_out/${T}_geo_$V.log 2>&1 || exit 1
done
