#!/bin/bash
# Round-5 GPU step: selected GPU tests (-k expr; "all" = every gpu test),
# then optionally the low-load latency probe.  Each GPU step has its own time
# limit; the script stops at the first failure.
#   tools/r5_gpu.sh TAG [KEXPR] [probe]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
K=${2:-}
if [ -n "$K" ]; then
  if [ "$K" = "all" ]; then KA=(); else KA=(-k "$K"); fi
  timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu "${KA[@]}" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  tail -5 gpurun_out/pytest_$TAG.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
fi
if [ "${3:-}" = "probe" ]; then
  timeout -k 10 400 python -u tools/latency_probe.py > gpurun_out/latency_$TAG.json 2> gpurun_out/latency_$TAG.err
  rc=$?
  tail -3 gpurun_out/latency_$TAG.err
  [ $rc -eq 0 ] || exit $rc
  python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/latency_{sys.argv[1]}.json"))
for cfg in ("go_default", "go_default_launch", "plain"):
    for route in ("small_route", "device_layer"):
        x = d[cfg][route]
        print(cfg, route, {k: round(v["p50_us"], 1) for k, v in x.items()})
c = d["c5_proxy"]
print("c5", {k: round(v["p50_us"], 1) for k, v in c["per_check"].items()}, "commit path", round(c["primary_commit_path_us"]["p50_us"], 1))
PY
fi
