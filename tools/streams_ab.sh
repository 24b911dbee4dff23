#!/bin/bash
# Batches in flight (--streams) A/B on one box, optionally with the
# diagnostic s^-1 reuse (DIAG=1: MBFT_DIAG_REUSE_WINV, the s^-1 stage's share).
set -o pipefail
for s in ${STREAMS:-1 2 3}; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --streams $s --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/streams_ab_$s$SUF.json 2> gpurun_out/streams_ab_$s$SUF.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/streams_ab_$s$SUF.json'));print('$s$SUF', d['ms_per_step'], d['kernel_ms'])"
done
