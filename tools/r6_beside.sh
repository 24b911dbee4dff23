#!/bin/bash
# Round 6: resident kernel beside 256K flat batches -- server count and poll
# back-off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6n}
mkdir -p $O
for rep in 1 2; do
for cfg in "16 1" "16 8" "16 32" "4 1" "8 8"; do
  set -- $cfg
  MBFT_RESIDENT_SERVERS=$1 MBFT_RESIDENT_POLL_SLEEP=$2 timeout -k 10 300 python3 tools/beside_probe.py >> $O/beside.jsonl 2>> $O/beside.err || { tail -20 $O/beside.err; exit 1; }
done
done
cat $O/beside.jsonl
