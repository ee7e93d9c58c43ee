# PMC breakdown of k_bp on the headline workload (one pass, 8 SQ + 1 GRBM counters)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bppmc -o run -- python3 $GRAFT_REPO_ROOT/tools/bp_only.py > $GRAFT_REPO_ROOT/gpurun_out/bppmc.log 2>&1
