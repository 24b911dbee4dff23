#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6q}
mkdir -p $O
export MBFT_RESIDENT_IDLE_US=1000000 MBFT_RESIDENT_LIFE_MS=5000
for s in 1 16; do
  MBFT_RESIDENT_SERVERS=$s timeout -k 10 300 python3 tools/launch_probe.py >> $O/launch.jsonl 2>> $O/launch.err || { tail -20 $O/launch.err; exit 1; }
done
cat $O/launch.jsonl
