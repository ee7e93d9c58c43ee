# bench --depth: the context / e2e / distributed GPU tests, headline-only bench lines at depth 2 and
# depth 1 (interleaved, twice), the 2-rank --share-gpu rehearsal at depth 2
set -o pipefail
T=${1:-r5s}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
NOLEGS="--no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress --no-gather-leg --no-geometries --no-sensitivity"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_context_reuse.py \
  tests/test_gpu_e2e.py tests/test_gpu_distributed.py tests/test_gpu_bench_parity.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  for d in 2 1; do
    timeout -k 10 300 python -u bench.py $NOLEGS --depth $d >> gpurun_out/${T}_bench_d$d.log 2>> gpurun_out/${T}_bench.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 > gpurun_out/${T}_rehearse2.log 2> gpurun_out/${T}_rehearse2.err
