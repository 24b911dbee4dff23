#!/bin/bash
# Round 6: the resident stream's kind against C2 interference -- lowest
# priority (default), CU-masked (round 5), and lowest priority with a longer
# lifetime; tools/resident_ab.py each, alternated twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6f
mkdir -p $O
for rep in 1 2; do
for cfg in "low 0 20" "cumask 1 20" "low200 0 200"; do
  set -- $cfg
  MBFT_RESIDENT_CUMASK=$2 MBFT_RESIDENT_LIFE_MS=$3 timeout -k 10 300 python3 tools/resident_ab.py --tag "$1" >> $O/ab.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
done
done
echo "[r6f] done"
