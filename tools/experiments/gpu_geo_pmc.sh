# PMC passes over the geometry legs (tools/experiments/geo_bench.py: 20 kHz bpt 2, 12 kHz bpt 10),
# each its own run as tools/gpu_pmc_r3.sh does for the headline; JSON summaries stamped with this
# tree's FT8_BUILD_ID.   usage: bash tools/gpu_geo_pmc.sh TAG -> gpurun_out/TAG_geo_pmc{,2,_traffic}.json
set -o pipefail
T=${1:-geopmc}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_gsq -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_gsq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_gsq2 -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_gsq2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_gfetch -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_gfetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_gwrite -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_gwrite.log 2>&1 &&
cd $R && python3 tools/pmc_sq_json.py gpurun_out/${T}_gsq gpurun_out/${T}_geo_pmc.json "rocprofv3 SQ/GRBM pass of tools/experiments/geo_bench.py, tools/gpu_geo_pmc.sh" &&
python3 tools/pmc_sq_json.py gpurun_out/${T}_gsq2 gpurun_out/${T}_geo_pmc2.json "rocprofv3 SQ LDS/SALU/VMEM pass of tools/experiments/geo_bench.py, tools/gpu_geo_pmc.sh" &&
python3 tools/pmc_traffic.py gpurun_out/${T}_gfetch gpurun_out/${T}_gwrite gpurun_out/${T}_geo_pmc_traffic.json
