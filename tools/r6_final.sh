#!/bin/bash
# Round 6 final measurement: the whole GPU suite, smoke(), the driver's bench
# command, a rocprofv3 kernel-trace pass of the headline loop (judged by its
# exit status), then the PMC passes over k_verify at the benched windows
# (counters in runs of their own).  Each GPU step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail.json > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
wc -c $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 bench.py --steps 20 --no-extra-lines --no-adversarial --c3-requests 0 --no-cpu-baseline --detail-out $O/kt_detail.json > $O/kt_bench.json 2> $O/kt.err || { echo "[r6_final] trace run failed"; tail -20 $O/kt.err; exit 1; }
K=$(find $O/kt -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$K" > $O/kernel_trace_summary.json || exit 1
cp "$(find $O/kt -name "*kernel_stats.csv" | head -1)" $O/kernel_stats.csv
rm -f "$K"
WINDOWS="29,29" bash tools/pmc_round.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_summarize.py gpurun_out/pmc > $O/pmc_w29_29.json || exit 1
echo "[r6_final] done"
