#!/bin/bash
# C3 line with the message layer's stage trace (MBFT_STAGE_TRACE), bench
# without the other extra lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1
MBFT_STAGE_TRACE=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-adversarial --no-extra-lines --no-cpu-baseline --no-peak-run > gpurun_out/c3_$TAG.json 2> gpurun_out/c3_$TAG.err
rc=$?
grep "mbft validate\|mbft calls" gpurun_out/c3_$TAG.err | tail -6
python3 -c "import json; d=json.load(open('gpurun_out/c3_$TAG.json')); print('C3 M msgs/s', d['c3_usig_streams']['messages_per_s']/1e6)"
exit $rc
