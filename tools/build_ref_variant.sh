# Build libft8hip.so from the csrc sources of an earlier commit, for same-box A/B runs against the
# current build:  bash tools/build_ref_variant.sh NAME COMMIT  ->  variants/NAME.so
# The sources are taken with `git archive` into a scratch directory and built with their own
# Makefile; the library keeps that commit's FT8_BUILD_ID, so the binding loads it only with
# FT8HIP_ALLOW_STALE=1 (the A/B tooling), never as the shipped build.
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d /tmp/ft8ref.XXXXXX)
git archive "$2" ft8_demodulator_amd/csrc include | tar -x -C "$T"
make -s -j8 -C "$T/ft8_demodulator_amd/csrc" 2>&1 | grep -v packed-fp32 || true
mkdir -p variants
cp "$T/ft8_demodulator_amd/lib/libft8hip.so" "variants/$1.so"
rm -rf "$T"
echo "variants/$1.so  (csrc of $2)"
