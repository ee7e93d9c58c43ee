# Barrier-race check build: every source compiled with -DFT8_RACE_CHECK (ft8_internal.h
# FT8_RACE_PROLOGUE: LDS filled with a sentinel, one wave per workgroup started late) and linked
# to variants/RACE.so, whose FT8_BUILD_ID carries "+variant-RACE" (the binding loads it only with
# FT8HIP_ALLOW_STALE=1).  Run the GPU suite on it:
#   FT8HIP_LIB=$PWD/variants/RACE.so FT8HIP_ALLOW_STALE=1 python -m pytest tests -m gpu
set -e
cd "$(dirname "$0")/../ft8_demodulator_amd/csrc"
mkdir -p ../../variants ../../build/race
SRC_ID=$(make -s -p 2>/dev/null | sed -n "s/^SRC_ID := //p" | head -1)
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result -DFT8_RACE_CHECK"
for s in stft stft3840 sync bp tx subtract drift; do
  EXTRA=$(make -s -p 2>/dev/null | sed -n "s/^EXTRA_$s := //p" | head -1)
  /opt/rocm/bin/hipcc $BASE $EXTRA -c $s.hip -o ../../build/race/$s.o 2>&1 | grep -v packed-fp32 || true &
done
/opt/rocm/bin/hipcc $BASE "-DFT8_BUILD_ID=\"$SRC_ID+variant-RACE:all\"" "-DFT8_BUILD_FLAGS=\"variant RACE: -DFT8_RACE_CHECK\"" \
  -c capi.hip -o ../../build/race/capi.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../variants/RACE.so $(for s in capi stft stft3840 sync bp tx subtract drift; do echo ../../build/race/$s.o; done)
echo variants/RACE.so
