# Kernel + memory-copy trace of StreamDecoder at depth D.  usage: bash tools/experiments/gpu_stream_trace2.sh TAG D
set -o pipefail
T=${1:-r5stream}
D=${2:-2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/${T}_trace -o run -- python3 $R/tools/experiments/stream_trace2.py $D > $R/gpurun_out/${T}.log 2>&1
