#!/bin/bash
# Quick GPU check: selected tests (-k expr), a short bench without the extra
# lines, and its kernel trace.  Each GPU step has its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/pytest_q_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_q_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_q_$TAG.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-adversarial --c3-requests 0 --no-extra-lines --no-cpu-baseline > gpurun_out/bench_q_$TAG.json 2> gpurun_out/bench_q_$TAG.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_q_$TAG -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/bench_qp_$TAG.json 2> gpurun_out/bench_qp_$TAG.err
rc=$?
[ $rc -eq 0 ] && python3 tools/trace_summary.py gpurun_out/prof_q_$TAG/kt_kernel_trace.csv > gpurun_out/kt_q_$TAG.json
python3 - "$TAG" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/bench_q_{t}.json"))
print("value", round(d["value"] / 1e6, 1), "M/s  ms/step", round(d["ms_per_step"], 4), " k_verify", round(d["kernel_ms"]["k_verify"], 4),
      " dev p50", round(d["p50_batch_latency_device_ms"], 4), " frac", round(d["roofline"]["frac"], 4))
PY
echo rc=$rc
exit $rc
