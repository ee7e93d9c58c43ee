# Round-4 final pass: GPU tests, smoke, PMC passes (build-stamped, placed in the box's profiles/ so
# the bench line reads this build's counters), the bench line, the headline kernel trace, the
# subtract-leg profile, the GPU suite on the barrier-race check build, the 2-rank rehearsal.
#   usage: bash tools/gpu_r4final.sh TAG   (then copy gpurun_out/TAG_pmc*.json into profiles/ here)
set -o pipefail
T=${1:-r4f}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
bash tools/gpu_pmc_r3.sh ${T} &&
cd $R && cp gpurun_out/${T}_pmc.json gpurun_out/${T}_pmc2.json gpurun_out/${T}_pmc_traffic.json profiles/ &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err &&
bash tools/gpu_prof.sh ${T} &&
bash tools/gpu_sub_prof.sh ${T} &&
cd $R && FT8HIP_LIB=$R/variants/RACE.so FT8HIP_ALLOW_STALE=1 timeout -k 10 900 python -u -m pytest tests -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_race_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpu --steps 10 --warmup 3 > gpurun_out/${T}_rehearse2.log 2> gpurun_out/${T}_rehearse2.err
