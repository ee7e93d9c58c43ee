# Round-5 pass C: new tests first, the GPU suite, same-box A/B against the round-4 library
# (tools/gpu_r5b.sh's legs), then the suite on the barrier-race check build.
set -o pipefail
T=${1:-r5c}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -rP --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_context_reuse.py tests/test_gpu_race_control.py "tests/test_gpu_tx.py::test_subtract_clean_signal_residual" \
  tests/test_gpu_harness.py > gpurun_out/${T}_new.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
for r in 1 2; do
  for L in R4 HEAD; do
    if [ $L = R4 ]; then LIB=$R/variants/R4.so; else LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; fi
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/sub_bench.py > gpurun_out/${T}_sub_${L}_$r.log 2>&1 || exit 1
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py > gpurun_out/${T}_geo_${L}_$r.log 2>&1 || exit 1
  done
done &&
timeout -k 10 600 python -u tools/ab_variants.py $R/variants/R4.so $R/ft8_demodulator_amd/lib/libft8hip.so > gpurun_out/${T}_ab.log 2>&1 &&
FT8HIP_LIB=$R/variants/RACE.so FT8HIP_ALLOW_STALE=1 timeout -k 10 900 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_race_tests.log 2>&1
