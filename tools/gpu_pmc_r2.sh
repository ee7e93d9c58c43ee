# PMC passes over the headline workload (tools/bp_only.py, 256 slots, config 3), each its own run:
# SQ/GRBM issue counters, then FETCH_SIZE, then WRITE_SIZE (gfx950: separate passes).
# usage: bash tools/gpu_pmc_r2.sh TAG   -> gpurun_out/TAG_{sq,fetch,write}/...
set -o pipefail
T=${1:-r2pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/${T}_counters.txt 2>&1 ;
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sq -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_write.log 2>&1
