# Context stream order (capi.hip StreamOrder): the context-reuse GPU tests on the in-tree build, the
# alternating-streams test on variants/O.so (the committed build without the order: expected to
# fail), then two contexts on two streams against one stream (tools/experiments/two_stream.py)
set -o pipefail
T=${1:-r5r}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_context_reuse.py \
  tests/test_gpu_e2e.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
FT8HIP_LIB=$R/variants/O.so FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_context_reuse.py -k alternating > gpurun_out/${T}_control_O.log 2>&1
echo "control exit $?" >> gpurun_out/${T}_control_O.log
timeout -k 10 300 python -u tools/experiments/two_stream.py > gpurun_out/${T}_two_stream.log 2>&1
