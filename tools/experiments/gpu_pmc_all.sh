# PMC passes over the headline workload (tools/bp_only.py, 256 slots, config 3), each its own run:
# SQ/GRBM issue counters (8 SQ + 1 GRBM), then FETCH_SIZE, then WRITE_SIZE (gfx950: separate passes)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sqpmc -o run -- python3 $GRAFT_REPO_ROOT/tools/bp_only.py > $GRAFT_REPO_ROOT/gpurun_out/sqpmc.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fpmc -o run -- python3 $GRAFT_REPO_ROOT/tools/bp_only.py > $GRAFT_REPO_ROOT/gpurun_out/fpmc.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/wpmc -o run -- python3 $GRAFT_REPO_ROOT/tools/bp_only.py > $GRAFT_REPO_ROOT/gpurun_out/wpmc.log 2>&1
