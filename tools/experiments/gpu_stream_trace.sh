# Kernel + memory-copy trace of the streaming leg (is the upload an SDMA copy or a blit kernel that
# waits for CUs?).  usage: bash tools/experiments/gpu_stream_trace.sh TAG
set -o pipefail
T=${1:-r3stream}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- python3 $R/tools/experiments/stream_probe.py > $R/gpurun_out/${T}.log 2>&1
