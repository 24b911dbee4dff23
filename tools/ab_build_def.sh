#!/bin/bash
# Build the WORKING TREE's C-ABI library with extra compiler definitions into
# minbft_amd/libminbft_amd_<TAG>.so (in-tree, travels to the GPU box), for
# same-box A/B (MBFT_LIB_PATH) or timing builds:
#   bash tools/ab_build_def.sh st "-DMBFT_SPLIT_TIMING"
set -e
TAG=$1; DEFS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d)
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wno-unused-result -I $ROOT/include $DEFS"
for f in $ROOT/minbft_amd/csrc/*.hip; do
  $H --offload-arch=gfx950 $F -c $f -o $OUT/$(basename $f .hip)_hip.o &
done
for f in $ROOT/minbft_amd/csrc/*.cpp; do
  $H $F -c $f -o $OUT/$(basename $f .cpp).o &
done
wait
$H --offload-arch=gfx950 -shared -fPIC -o "$ROOT/minbft_amd/libminbft_amd_$TAG.so" $OUT/*.o
rm -rf "$OUT"
echo "$ROOT/minbft_amd/libminbft_amd_$TAG.so"
