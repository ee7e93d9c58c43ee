# Round-5 final pass, part B: the headline kernel trace, the subtract-leg profile, the GPU suite on
# the barrier-race check build (variants/RACE.so, tools/build_race.sh), the 2-rank rehearsal.
set -o pipefail
T=${1:-r5_v3}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_prof.sh ${T} &&
bash tools/gpu_sub_prof.sh ${T} &&
cd $R && FT8HIP_LIB=$R/variants/RACE.so FT8HIP_ALLOW_STALE=1 timeout -k 10 900 python -u -m pytest tests -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_race_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 > gpurun_out/${T}_rehearse2.log 2> gpurun_out/${T}_rehearse2.err &&
# N = 1 with the per-step RCCL exchange inside the depth-2 timed loop (world-size-1 group)
timeout -k 10 300 python -u bench.py --gather --no-cpu --no-h2d --no-subtract --no-drift --no-bp-stress --no-gather-leg \
  --no-geometries --no-sensitivity > gpurun_out/${T}_gather_n1.json.log 2> gpurun_out/${T}_gather_n1.err
