# Drift-leg timing of several libraries, interleaved twice (no tests).
# usage: bash tools/gpu_drift_ab3.sh TAG lib1.so lib2.so ...   (paths relative to the repo)
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for k in 1 2; do
  for L in "$@"; do
    n=$(basename $L .so)
    FT8HIP_LIB=$R/$L FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --no-subtract --no-bp-stress --no-gather-leg > gpurun_out/${T}_${n}_$k.log 2>&1 || exit 1
  done
done
