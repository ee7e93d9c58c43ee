# multi-frame k_stft_pk (kPkFrames frames per workgroup, window in registers): the STFT / reftest /
# stage GPU tests on the in-tree build (next frame prefetched, 8 frames) and on variant PB (no
# prefetch), then the geometry legs interleaved: O (committed, one frame per workgroup), N (in-tree),
# PB, PB4 (no prefetch, 4 frames), PN4 (prefetch, 4 frames)
set -o pipefail
T=${1:-r5j}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stft.py \
  tests/test_gpu_reftests.py tests/test_gpu_stages.py > gpurun_out/${T}_tests.log 2>&1 || exit 1
FT8HIP_LIB=$R/variants/PB.so FT8HIP_ALLOW_STALE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stft.py \
  tests/test_gpu_reftests.py > gpurun_out/${T}_tests_PB.log 2>&1 || exit 1
for i in 1 2; do
  for V in O N PB PB4 PN4; do
    if [ $V = N ]; then LIB=$R/ft8_demodulator_amd/lib/libft8hip.so; else LIB=$R/variants/$V.so; fi
    FT8HIP_LIB=$LIB FT8HIP_ALLOW_STALE=1 timeout -k 10 300 python -u tools/experiments/geo_bench.py >> gpurun_out/${T}_geo_$V.log 2>&1 || exit 1
  done
done
