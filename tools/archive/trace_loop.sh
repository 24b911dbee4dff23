#!/bin/bash
# Kernel trace of a short bench run (timed-loop overlap analysis):
# gpurun_out/prof_loop_$TAG/, then tools/loop_timeline.py on it.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-loop}
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$TAG -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
