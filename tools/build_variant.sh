# Build an A/B variant of libft8hip.so with extra flags for one source file:
#   bash tools/build_variant.sh NAME FILE "FLAGS"      e.g.  bash tools/build_variant.sh B stft3840 "-DX=1"
# -> variants/NAME.so (every other object from the current in-tree build).  The variant's capi
# object carries FT8_BUILD_ID "<source id>+variant-NAME:FILE" and the extra flags, so the Python
# binding refuses it unless FT8HIP_ALLOW_STALE=1 (set by tools/gpu_ab.sh), and a variant can never
# pass for the shipped build.  Record the NAME -> FLAGS map next to the A/B log it produces.
set -e
cd "$(dirname "$0")/../ft8_demodulator_amd/csrc"
make -s
mkdir -p ../../variants ../../build/var
F=$2
EXTRA=$(make -s -p 2>/dev/null | sed -n "s/^EXTRA_$F := //p" | head -1)
SRC_ID=$(make -s -p 2>/dev/null | sed -n "s/^SRC_ID := //p" | head -1)
BASE="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result"
/opt/rocm/bin/hipcc $BASE $EXTRA $3 -c $F.hip -o ../../build/var/$1_$F.o
/opt/rocm/bin/hipcc $BASE "-DFT8_BUILD_ID=\"$SRC_ID+variant-$1:$F\"" "-DFT8_BUILD_FLAGS=\"variant $1: $F.hip $3\"" \
  -c capi.hip -o ../../build/var/$1_capi.o
OBJS=$(for s in capi stft stft3840 sync bp tx subtract drift; do
  if [ $s = $F ] || [ $s = capi ]; then echo ../../build/var/$1_$s.o; else echo ../../build/$s.o; fi; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../variants/$1.so $OBJS
echo "variants/$1.so  ($F.hip: $3)"
