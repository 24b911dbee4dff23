#!/bin/bash
# bench.py value vs timed-window length (warmup, steps): where does the
# measurement reach the sustained (power-capped) steady state?
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
for ws in "3 20" "20 200" "100 500" "200 1000"; do
  set -- $ws
  timeout -k 10 300 python bench.py --warmup $1 --steps $2 --latency-reps 3 --no-cpu-baseline --no-peak-run \
    > gpurun_out/sweep/w$1_s$2.json 2> gpurun_out/sweep/w$1_s$2.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/w$1_s$2.json'));print('warmup $1 steps $2: %.1fM ms/step %.4f'%(d['value']/1e6,d['ms_per_step']))"
done
