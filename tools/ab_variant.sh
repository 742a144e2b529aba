# Build the CURRENT tree's libpcx.so (or git revision REV's) with extra compiler flags into
# ab/NAME/libpcx.so.
# usage: [REV=HEAD~1] bash tools/ab_variant.sh NAME "-DFOO=1 -DBAR=2"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/ab/$NAME
rm -rf "$D" && mkdir -p "$D/src"
if [ -n "$REV" ]; then
  git -C "$ROOT" archive "$REV" pyconsensus_amd/csrc include | tar -x -C "$D/src"
else
  tar -C "$ROOT" -cf - pyconsensus_amd/csrc include | tar -x -C "$D/src"
fi
rm -rf "$D/src/pyconsensus_amd/csrc/build"
make -s -j8 -C "$D/src/pyconsensus_amd/csrc" CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function -I$D/src/include $FLAGS"
mv "$D/src/pyconsensus_amd/libpcx.so" "$D/libpcx.so"
rm -rf "$D/src"
echo "$D/libpcx.so"
