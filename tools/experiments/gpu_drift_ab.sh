# Drift-leg A/B: gpu tests, then bench.py's drift leg (headline + drift only) with a variant library
# and the in-tree build, interleaved twice.  usage: bash tools/gpu_drift_ab.sh TAG variants/OLD.so
set -o pipefail
T=${1:-r3drift}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
for k in 1 2; do
  FT8HIP_LIB=$R/$2 FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --no-subtract --no-bp-stress --no-gather-leg > gpurun_out/${T}_old$k.log 2>&1 &&
  timeout -k 10 300 python -u bench.py --no-cpu --no-h2d --no-subtract --no-bp-stress --no-gather-leg > gpurun_out/${T}_new$k.log 2>&1 || exit 1
done
