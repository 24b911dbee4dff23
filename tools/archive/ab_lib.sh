#!/bin/bash
# Same-box A/B of library builds: bench.py alternating between the in-tree
# library ("new") and minbft_amd/libminbft_amd_<TAG>.so for each TAG given.
#   bash tools/ab_lib.sh base [other ...]      (extra bench args via BENCH_ARGS)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for rep in 1 2; do
  for tag in new "$@"; do
    if [ "$tag" = new ]; then L=""; else L="$PWD/minbft_amd/libminbft_amd_$tag.so"; fi
    MBFT_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-peak-run --latency-reps 3 $BENCH_ARGS > gpurun_out/ab/${tag}_$rep.json 2> gpurun_out/ab/${tag}_$rep.err || { tail -n 20 gpurun_out/ab/${tag}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ab/${tag}_$rep.json'));print('$tag rep $rep value %.1fM'%(d['value']/1e6),'k_verify %.4f ms'%d['kernel_ms']['k_verify'])"
  done
done
