#!/bin/bash
# Round 6: the s^-1 stage's forms in the C2 loop, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6k}
mkdir -p $O
for rep in 1 2; do
  for cfg in "default 3" "local 3" "local 2" "local 1" "levels 3"; do
    set -- $cfg
    if [ $1 = default ]; then unset MBFT_NINV; else export MBFT_NINV=$1; fi
    timeout -k 10 300 python3 tools/steady_ab.py --streams $2 --tag "$1_s$2" >> $O/ninv.jsonl 2>> $O/ninv.err || { tail -20 $O/ninv.err; exit 1; }
  done
done
unset MBFT_NINV
cat $O/ninv.jsonl
