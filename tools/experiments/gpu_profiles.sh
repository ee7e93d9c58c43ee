# rocprofv3 kernel statistics of the bench's headline workload alone and of the drift leg alone,
# so each kernel's average matches the bench line's HIP-event figure for the same launches.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profm -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress > $GRAFT_REPO_ROOT/gpurun_out/profm.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/profd -o run -- python3 $GRAFT_REPO_ROOT/tools/experiments/drift_bench.py > $GRAFT_REPO_ROOT/gpurun_out/profd.log 2>&1
