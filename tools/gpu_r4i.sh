# Round-4 pass I: the STFT tests (the int16 == float32 case of the packed plans) and an interleaved
# A/B of k_stft3840p run lengths (variants/CH4.so, CH8.so, CH12.so against this build's 6).
#   usage: bash tools/gpu_r4i.sh TAG
set -o pipefail
T=${1:-r4i}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v -rP --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stft.py > gpurun_out/${T}_stft_tests.log 2>&1
rc=$?
echo "stft_tests rc=$rc" > gpurun_out/${T}_steps.txt
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 800 python -u tools/ab_variants.py $R/ft8_demodulator_amd/lib/libft8hip.so $R/variants/CH4.so $R/variants/CH8.so $R/variants/CH12.so > gpurun_out/${T}_chunk_ab.log 2>&1
echo "ab rc=$?" >> gpurun_out/${T}_steps.txt
