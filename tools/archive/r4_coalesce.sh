#!/bin/bash
# Check coalescing (round 4): its GPU tests, the msgdev tests it touches, and
# the C3 line with the Go-wiring variants.
set -o pipefail
O=gpurun_out
TAG=${1:-co}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_check_coalesce.py tests/test_gpu_msgdev.py > $O/pytest_co_$TAG.log 2>&1 || { tail -40 $O/pytest_co_$TAG.log; exit 1; }
tail -2 $O/pytest_co_$TAG.log
timeout -k 10 400 python -u tools/c3_probe.py 16384 > $O/c3_co_$TAG.json 2> $O/c3_co_$TAG.err || { tail -20 $O/c3_co_$TAG.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c3_co_$TAG.json')); g=d['go_wiring']
print('c3', round(d['messages_per_s']/1e6,1), 'go', round(g['messages_per_s']/1e6,1), {k: (round(v['messages_per_s']/1e6,1), v['device_passes_per_run'], round(v['mean_messages_per_pass'])) for k,v in g['coalesced'].items()})"
