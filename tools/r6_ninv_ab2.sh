#!/bin/bash
# Round 6: the one-launch s^-1's forms (per block / per wave, chain length)
# in the C2 loop with 3 and 1 caller streams.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6l}
mkdir -p $O
export MBFT_NINV=local
for cfg in "block 8 3" "wave 16 3" "wave 8 3" "block 4 3" "block 8 1" "wave 16 1" "wave 8 1" "wave 4 3"; do
  set -- $cfg
  MBFT_NINV_FORM=$1 MBFT_NINV_PER=$2 timeout -k 10 300 python3 tools/steady_ab.py --streams $3 --tag "$1_$2_s$3" >> $O/ninv.jsonl 2>> $O/ninv.err || { tail -20 $O/ninv.err; exit 1; }
done
cat $O/ninv.jsonl
