# usage: bash pmc_variants.sh TAG VARIANT...   (variants/VARIANT.so, two SQ passes each)
set -o pipefail
T=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
export FT8HIP_ALLOW_STALE=1
for V in "$@"; do
  export FT8HIP_LIB=$R/variants/$V.so
  (cd /tmp && export TMPDIR=/tmp &&
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_${V}_sq -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_${V}_sq.log 2>&1 &&
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_${V}_sq2 -o run -- python3 $R/tools/bp_only.py > $R/gpurun_out/${T}_${V}_sq2.log 2>&1) || exit 1
  (cd $R && python3 tools/pmc_sq_json.py gpurun_out/${T}_${V}_sq gpurun_out/${T}_${V}_pmc.json "variant $V" &&
   python3 tools/pmc_sq_json.py gpurun_out/${T}_${V}_sq2 gpurun_out/${T}_${V}_pmc2.json "variant $V") || exit 1
  rm -rf $R/gpurun_out/${T}_${V}_sq $R/gpurun_out/${T}_${V}_sq2
done
