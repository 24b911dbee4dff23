#!/bin/bash
# Round 6: the pooled resident servers -- GPU tests of the resident paths,
# then tools/resident_ab.py at several pool sizes and with the 3-wave build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_small_check.py tests/test_gpu_replies_go.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for cfg in "16 default" "64 default" "8 default" "16 w3" "32 w3"; do
  set -- $cfg
  if [ $2 = w3 ]; then L=minbft_amd/libminbft_amd_w3.so; else L=minbft_amd/libminbft_amd.so; fi
  MBFT_RESIDENT_SERVERS=$1 MBFT_LIB_PATH=$L timeout -k 10 300 python3 tools/resident_ab.py --tag "s$1_$2" >> $O/ab.jsonl 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
done
echo "[r6c] done"
