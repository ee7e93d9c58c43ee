# Build an A/B variant of libft8hip.so with extra flags for one source file:
#   bash tools/build_variant.sh NAME FILE "FLAGS"      e.g.  bash tools/build_variant.sh B bp "-DBP_WAVES_PER_EU=5"
# -> variants/NAME.so (every other object from the current in-tree build)
set -e
cd "$(dirname "$0")/../ft8_demodulator_amd/csrc"
make -s
mkdir -p ../../variants ../../build/var
F=$2
EXTRA=$(make -s -p 2>/dev/null | sed -n "s/^EXTRA_$F := //p" | head -1)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result $EXTRA $3 -c $F.hip -o ../../build/var/$1_$F.o
OBJS=$(for s in capi stft stft3840 sync bp tx subtract drift; do if [ $s = $F ]; then echo ../../build/var/$1_$F.o; else echo ../../build/$s.o; fi; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../../variants/$1.so $OBJS
echo variants/$1.so
