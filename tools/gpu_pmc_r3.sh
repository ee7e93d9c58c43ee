# PMC passes over the headline workload (tools/bp_only.py, 256 slots, config 3), each its own run:
# SQ/GRBM issue counters, then FETCH_SIZE, then WRITE_SIZE (gfx950: separate passes), then the JSON
# summaries for bench.py, stamped with this tree's FT8_BUILD_ID.
# usage: bash tools/gpu_pmc_r3.sh TAG   -> gpurun_out/TAG_{sq,fetch,write}/..., gpurun_out/TAG_pmc*.json
set -o pipefail
T=${1:-r3pmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sq -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sq2 -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_sq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_write.log 2>&1 &&
cd $R && python3 tools/pmc_sq_json.py gpurun_out/${T}_sq gpurun_out/${T}_pmc.json "rocprofv3 SQ/GRBM pass of tools/bp_only.py (256 slots, config 3), tools/gpu_pmc_r3.sh" &&
python3 tools/pmc_sq_json.py gpurun_out/${T}_sq2 gpurun_out/${T}_pmc2.json "rocprofv3 SQ LDS/SALU/VMEM pass of tools/bp_only.py (256 slots, config 3), tools/gpu_pmc_r3.sh" &&
python3 tools/pmc_traffic.py gpurun_out/${T}_fetch gpurun_out/${T}_write gpurun_out/${T}_pmc_traffic.json
