# Build libpcx.so of git revision REV into ab/REV/libpcx.so (for A/B runs: PCX_LIB=ab/REV/libpcx.so).
# usage: bash tools/ab_build.sh REV
set -e
REV=$1
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/ab/$REV
rm -rf "$D" && mkdir -p "$D/src"
git -C "$ROOT" archive "$REV" pyconsensus_amd/csrc include | tar -x -C "$D/src"
make -s -j8 -C "$D/src/pyconsensus_amd/csrc"
mv "$D/src/pyconsensus_amd/libpcx.so" "$D/libpcx.so"
rm -rf "$D/src"
echo "$D/libpcx.so"
