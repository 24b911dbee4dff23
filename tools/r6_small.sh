#!/bin/bash
# Round 6: the small route's host work -- SHA lanes on this host's CPU, the
# GPU tests of the changed paths, then the low-load windows with the stage
# trace (512-message windows) and without (every size).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6j}
mkdir -p $O
for L in 1 2 3 4; do echo "lanes $L"; timeout -k 5 60 tools/sha_bench_l$L; done > $O/sha_lanes.txt 2>&1
cat $O/sha_lanes.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_small_check.py tests/test_gpu_msgdev.py tests/test_gpu_multi.py tests/test_gpu_multi_msg.py tests/test_gpu_check_coalesce.py tests/test_gpu_authen.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MBFT_STAGE_TRACE=1 LOWLOAD_SIZES=512 timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload_trace.json 2> $O/lowload_trace.err || { tail -20 $O/lowload_trace.err; exit 1; }
grep "mbft small calls\|mbft stage\]\|check small" $O/lowload_trace.err | tail -12
timeout -k 10 300 python3 tools/lowload_probe.py > $O/lowload.json 2> $O/lowload.err || { tail -20 $O/lowload.err; exit 1; }

if [ -n "$R6CLK" ]; then
  MBFT_LIB_PATH=minbft_amd/libminbft_amd_clk.so timeout -k 10 300 python3 tools/clock_stamp_probe.py > $O/clock.jsonl 2> $O/clock.err || { tail -20 $O/clock.err; exit 1; }
  MBFT_DIAG_REUSE_WINV=1 MBFT_LIB_PATH=minbft_amd/libminbft_amd_clk.so timeout -k 10 300 python3 tools/clock_stamp_probe.py >> $O/clock.jsonl 2>> $O/clock.err || { tail -20 $O/clock.err; exit 1; }
  cat $O/clock.jsonl
fi
echo "[r6_small] done"
