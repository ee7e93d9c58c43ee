# k_bp ticket order (rank-major, weakest first): the decode / BP / context GPU tests on the in-tree
# build, then the headline step interleaved against variants/BO0.so (slot-major order), 4 rounds
set -o pipefail
T=${1:-r5q}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bench_parity.py \
  tests/test_gpu_e2e.py tests/test_gpu_stages.py tests/test_gpu_context_reuse.py tests/test_gpu_reftests.py \
  tests/test_gpu_subtract_oracle.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 600 python -u tools/ab_variants.py $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/BO0.so >> gpurun_out/${T}_ab.log 2>&1 || exit 1
done
