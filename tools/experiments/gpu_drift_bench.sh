set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_drift.py tests/test_gpu_stft.py tests/test_gpu_e2e.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/db_t.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pdb6 -o run -- python3 $GRAFT_REPO_ROOT/tools/experiments/drift_bench.py > $GRAFT_REPO_ROOT/gpurun_out/pdb6.log 2>&1
