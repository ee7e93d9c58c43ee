# Round-4 pass G: the dev build against this one -- second-pass digests (bit-identity), STFT /
# reference-geometry / subtract tests on the dev build, the geometry legs and the subtract leg
# interleaved, and a kernel trace + one SQ pass of the geometry legs on the dev build.
#   usage: bash tools/gpu_r4g.sh TAG    (variants/DEV.so = the dev build)
set -o pipefail
T=${1:-r4g}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  local name=$1 to=$2
  shift 2
  timeout -k 10 "$to" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/${T}_steps.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
MAIN=$R/ft8_demodulator_amd/lib/libft8hip.so
DEV=$R/variants/DEV.so
PYT="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
FT8HIP_LIB=$MAIN FT8HIP_ALLOW_STALE=1 run digest_main 300 python -u tools/experiments/sub_digest.py
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run digest_dev 300 python -u tools/experiments/sub_digest.py
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run devtests 600 $PYT -x tests/test_gpu_stft.py tests/test_gpu_reftests.py tests/test_gpu_e2e.py tests/test_gpu_tx.py tests/test_gpu_subtract_oracle.py tests/test_gpu_drift.py
for i in 1 2; do
  FT8HIP_LIB=$MAIN FT8HIP_ALLOW_STALE=1 run geo_main$i 300 python -u tools/experiments/geo_bench.py
  FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run geo_dev$i 300 python -u tools/experiments/geo_bench.py
done
FT8HIP_LIB=$MAIN FT8HIP_ALLOW_STALE=1 run sub_main 300 python -u tools/experiments/sub_bench.py
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 run sub_dev 300 python -u tools/experiments/sub_bench.py
cd /tmp && export TMPDIR=/tmp
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_geo_trace -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_geo_trace.log 2>&1 || exit 1
FT8HIP_LIB=$DEV FT8HIP_ALLOW_STALE=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/${T}_geo_sq -o run -- python3 $R/tools/experiments/geo_bench.py > $R/gpurun_out/${T}_geo_sq.log 2>&1 || exit 1
cd $R && python3 tools/pmc_sq_json.py gpurun_out/${T}_geo_sq gpurun_out/${T}_geo_pmc.json "rocprofv3 SQ/GRBM pass of the geometry legs (tools/experiments/geo_bench.py), dev build"
