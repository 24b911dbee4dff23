#!/bin/bash
# C3 device message layer under rocprofv3 --kernel-trace --memory-copy-trace:
# copy / kernel timeline of the last validate call (tools/copy_timeline.py).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-c3tl}
MBFT_STAGE_TRACE=1 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace \
  --output-format csv -d gpurun_out/$TAG -o tl -- python3 tools/c3_probe.py 16384 \
  > gpurun_out/$TAG.json 2> gpurun_out/$TAG.err || { tail -20 gpurun_out/$TAG.err; exit 1; }
python3 tools/copy_timeline.py gpurun_out/$TAG/tl 8 > gpurun_out/$TAG.txt || exit 1
tail -80 gpurun_out/$TAG.txt
