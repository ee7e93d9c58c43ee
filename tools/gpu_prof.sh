# rocprofv3 kernel trace + stats of the headline workload alone (no CPU leg, no side legs): warm-up,
# timed loop and the per-kernel back-to-back re-launches; tools/trace_steps.py reconciles the trace
# with the bench line printed by the same run.  usage: bash tools/gpu_prof.sh TAG
set -o pipefail
T=${1:-r2}
shift
EXTRA="$*"   # extra bench.py flags (e.g. --depth 1 --no-single-call)
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_prof -o run -- python3 $R/bench.py --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress --no-gather-leg --no-geometries --no-sensitivity $EXTRA > $R/gpurun_out/${T}_prof.log 2>&1 &&
cd $R && python3 tools/trace_steps.py gpurun_out/${T}_prof/run_kernel_trace.csv gpurun_out/${T}_prof.log -o gpurun_out/${T}_steps.json > /dev/null
