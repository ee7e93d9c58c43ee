# SQ issue counters of the drift leg's kernels (one pass, tools/experiments/drift_only.py).
# usage: bash tools/experiments/gpu_drift_pmc.sh TAG
set -o pipefail
T=${1:-r3drift}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sq -o run -- python3 $R/tools/experiments/drift_only.py > $R/gpurun_out/${T}_sq.log 2>&1 &&
cd $R && python3 tools/pmc_sq_json.py gpurun_out/${T}_sq gpurun_out/${T}_pmc.json "rocprofv3 SQ/GRBM pass of tools/experiments/drift_only.py (256 complex128 beacons)"
