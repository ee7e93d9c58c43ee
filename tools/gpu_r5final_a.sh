# Round-5 final pass, part A: GPU suite, smoke, the build-stamped PMC passes (copied into the box's
# profiles/ so the bench line reads this build's counters), the bench line.
#   usage: bash tools/gpu_r5final_a.sh TAG   (TAG r<round>_v<k>; copy gpurun_out/TAG_pmc*.json into profiles/ here)
set -o pipefail
T=${1:-r5_v3}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -rP --timeout 300 --timeout-method thread -m gpu > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
bash tools/gpu_pmc_r3.sh ${T} &&
cd $R && cp gpurun_out/${T}_pmc.json gpurun_out/${T}_pmc2.json gpurun_out/${T}_pmc_traffic.json profiles/ &&
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2> gpurun_out/${T}_bench.err
