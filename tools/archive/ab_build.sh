#!/bin/bash
# Build the C-ABI library as it was at git revision REV into
# minbft_amd/libminbft_amd_<TAG>.so (in-tree, so it travels to the GPU box),
# for same-box A/B timing:  MBFT_LIB_PATH=$PWD/minbft_amd/libminbft_amd_<TAG>.so python bench.py
#   bash tools/ab_build.sh REV TAG
set -e
REV=$1; TAG=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$(mktemp -d)
git -C "$ROOT" archive "$REV" minbft_amd/csrc include | tar -x -C "$SRC"
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wno-unused-result -I $SRC/include"
for f in $SRC/minbft_amd/csrc/*.hip; do
  $H --offload-arch=gfx950 $F -c $f -o $SRC/$(basename $f .hip)_hip.o &
done
for f in $SRC/minbft_amd/csrc/*.cpp; do
  $H $F -c $f -o $SRC/$(basename $f .cpp).o &
done
wait
$H --offload-arch=gfx950 -shared -fPIC -o "$ROOT/minbft_amd/libminbft_amd_$TAG.so" $SRC/*.o
rm -rf "$SRC"
echo "$ROOT/minbft_amd/libminbft_amd_$TAG.so"
