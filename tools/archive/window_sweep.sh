#!/bin/bash
# Comb-window sweep: parity on the golden vectors, then bench.py per (G, Q)
# window pair.  Each GPU step has its own time limit; stop at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread > gpurun_out/sweep/parity.log 2>&1 || { tail -20 gpurun_out/sweep/parity.log; exit 1; }
tail -n 2 gpurun_out/sweep/parity.log
LIST=${SWEEP:-16,16 20,20 22,22 24,24 26,26 26,22}
for gq in $LIST; do
  g=${gq%,*}; q=${gq#*,}
  echo "[sweep] G=$g Q=$q"
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --latency-reps 3 --g-window $g --q-window $q > gpurun_out/sweep/b_${g}_${q}.json 2> gpurun_out/sweep/b_${g}_${q}.err || { tail -20 gpurun_out/sweep/b_${g}_${q}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/sweep/b_${g}_${q}.json'));print('G',$g,'Q',$q,'value %.1fM'%(d['value']/1e6),'kverify %.3f ms'%d['kernel_ms']['k_verify'],'inv %.3f'%d['kernel_ms']['batched_inverse_span_overlapped'],'frac %.3f'%d['roofline']['frac'],'tables %.1f s'%d['table_build_s'])"
done
