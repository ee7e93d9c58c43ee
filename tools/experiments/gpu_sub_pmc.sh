# PMC breakdown of the subtract-and-redecode kernels (one pass, 8 SQ + 1 GRBM counters)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/subpmc -o run -- python3 $GRAFT_REPO_ROOT/tools/experiments/sub_bench.py > $GRAFT_REPO_ROOT/gpurun_out/subpmc.log 2>&1
