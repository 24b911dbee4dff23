#!/bin/bash
# Same-box A/B of environment settings: bench.py alternating between the
# given env assignments (each "NAME=VALUE[,NAME=VALUE]"), 2 reps each.
#   BENCH_ARGS="--g-window 16 --q-window 16" bash tools/ab_env.sh MBFT_VERIFY_SPECIALIZE=0 MBFT_VERIFY_SPECIALIZE=1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    tag=$(echo "$v" | tr ',=' '__')
    env $(echo "$v" | tr ',' ' ') timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-peak-run --latency-reps 10 $BENCH_ARGS > gpurun_out/ab/$tag.$rep.json 2> gpurun_out/ab/$tag.$rep.err || { tail -n 20 gpurun_out/ab/$tag.$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/$tag.$rep.json'));print('$v rep $rep value %.1fM'%(d['value']/1e6),'k_verify %.4f ms'%d['kernel_ms']['k_verify'])"
  done
done
