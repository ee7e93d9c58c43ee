# Pre-flight for a GPU call from the dev container: rebuild the library in-tree, make sure the
# Python binding accepts it (its FT8_BUILD_ID equals the tree's sources), then run gpurun.
#   bash tools/gpu_call.sh TIMEOUT 'command' > log
set -e
cd "$(dirname "$0")/.."
make -s -C ft8_demodulator_amd/csrc -j8 2>&1 | grep -v packed-fp32-ops || true
python3 -c "import sys; sys.path.insert(0, '.'); from ft8_demodulator_amd import _lib; _lib.lib(); print('library current:', _lib.lib().ft8_build_id().decode())"
exec /usr/local/graft/bin/gpurun --timeout "$1" -- "$2"
