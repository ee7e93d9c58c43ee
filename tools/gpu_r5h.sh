# 640-thread k_stft_pk<9600> (every stage's butterfly count a multiple of 640 or within 6 % of it):
# the STFT / reftest / stage GPU tests on the current build, then the geometry legs interleaved
# against variants/O.so (the committed csrc)
set -o pipefail
T=${1:-r5h}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stft.py \
  tests/test_gpu_reftests.py tests/test_gpu_stages.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  FT8HIP_LIB=$R/variants/O.so FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py >> gpurun_out/${T}_geo_O.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/experiments/geo_bench.py >> gpurun_out/${T}_geo_N.log 2>&1 || exit 1
done
