#!/bin/bash
# Round 6: what costs the flat batches beside the resident verifier -- the
# live kernel with no posts (idle exit 1 s), the calls through the launch
# path (resident off), both.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6o}
mkdir -p $O
for rep in 1 2; do
for m in resident_idle calls_only resident_calls; do
  BESIDE_MODE=$m MBFT_RESIDENT_IDLE_US=1000000 MBFT_RESIDENT_LIFE_MS=2000 timeout -k 10 300 python3 tools/beside_probe.py >> $O/beside.jsonl 2>> $O/beside.err || { tail -20 $O/beside.err; exit 1; }
done
done
cat $O/beside.jsonl
