#!/bin/bash
# Build the WORKING TREE's C-ABI library with extra compiler definitions into
# minbft_amd/libminbft_amd_<TAG>.so (in-tree, travels to the GPU box), for
# same-box A/B with tools/ab_lib.sh:
#   bash tools/ab_build_def.sh nt "-DMBFT_GATHER_CPOL=2"
set -e
TAG=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d)
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wno-unused-result -I $ROOT/include $DEFS"
$H --offload-arch=gfx950 $F -c $ROOT/minbft_amd/csrc/kernels.hip -o $OUT/k.o &
for f in host der messages; do
  [ -f $ROOT/minbft_amd/csrc/$f.cpp ] && $H $F -c $ROOT/minbft_amd/csrc/$f.cpp -o $OUT/$f.o &
done
wait
$H --offload-arch=gfx950 -shared -fPIC -o "$ROOT/minbft_amd/libminbft_amd_$TAG.so" $OUT/*.o
rm -rf "$OUT"
echo "$ROOT/minbft_amd/libminbft_amd_$TAG.so"
