#!/bin/bash
# Round 6: the idle resident kernel's cost to flat batches against its
# server count and its stream kind.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6p}
mkdir -p $O
export BESIDE_MODE=resident_idle MBFT_RESIDENT_IDLE_US=1000000 MBFT_RESIDENT_LIFE_MS=2000
for cfg in "1 0" "2 0" "16 0" "16 1" "1 1"; do
  set -- $cfg
  MBFT_RESIDENT_SERVERS=$1 MBFT_RESIDENT_CUMASK=$2 timeout -k 10 300 python3 tools/beside_probe.py | sed "s/^{/{\"cumask\": $2, /" >> $O/beside.jsonl 2>> $O/beside.err || { tail -20 $O/beside.err; exit 1; }
done
cat $O/beside.jsonl
