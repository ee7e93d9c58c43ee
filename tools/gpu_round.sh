set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/t9.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/b9.log 2> gpurun_out/b9.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof9 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-h2d > $GRAFT_REPO_ROOT/gpurun_out/p9.log 2>&1
