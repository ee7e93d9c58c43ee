# k_stft_pk<9600> pruned first stage (two nonzero inputs per butterfly): GPU tests, geometry legs vs O
# (variants/O.so = the committed build): STFT / reftest / stage / harness tests, three interleaved rounds
set -o pipefail
T=${1:-r5u}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stft.py \
  tests/test_gpu_reftests.py tests/test_gpu_stages.py tests/test_gpu_harness.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for V in O N; do
    if [ $V = N ]; then LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; else LIB=$R/variants/$V.so; fi
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py >> gpurun_out/${T}_geo_$V.log 2>&1 || exit 1
  done
done
