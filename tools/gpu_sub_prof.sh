# Config-4 second pass on evidence: the subtract-and-redecode bench leg alone
# (tools/experiments/sub_bench.py: 334 crowded slots, top-k K=300, 50 BP iterations, both passes)
# under a rocprofv3 kernel trace + stats, then FETCH_SIZE, WRITE_SIZE and one SQ/GRBM pass, each its
# own run; the JSON summaries carry this tree's FT8_BUILD_ID.
#   usage: bash tools/gpu_sub_prof.sh TAG  -> gpurun_out/TAG_sub_{trace,fetch,write,sq}/, TAG_sub_*.json
set -o pipefail
T=${1:-r4}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
SRC="the subtract_redecode bench leg (tools/experiments/sub_bench.py: 334 slots, top-k K=300, 50 iterations, 4 launches)"
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_sub_trace -o run -- python3 $R/tools/experiments/sub_bench.py > $R/gpurun_out/${T}_sub_trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sub_fetch -o run -- python3 $R/tools/experiments/sub_bench.py > $R/gpurun_out/${T}_sub_fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sub_write -o run -- python3 $R/tools/experiments/sub_bench.py > $R/gpurun_out/${T}_sub_write.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_sub_sq -o run -- python3 $R/tools/experiments/sub_bench.py > $R/gpurun_out/${T}_sub_sq.log 2>&1 &&
cd $R && python3 tools/pmc_traffic.py gpurun_out/${T}_sub_fetch gpurun_out/${T}_sub_write gpurun_out/${T}_sub_pmc_traffic.json "$SRC" &&
python3 tools/pmc_sq_json.py gpurun_out/${T}_sub_sq gpurun_out/${T}_sub_pmc.json "rocprofv3 SQ/GRBM pass of $SRC" &&
python3 tools/kernel_summary.py gpurun_out/${T}_sub_trace gpurun_out/${T}_sub_kernels.json "$SRC"
