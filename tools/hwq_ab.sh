#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) A/B on one
# box: the C3 line with the Go-wiring variants (many streams: 4 lanes x 3-4
# streams each), and the C2 headline.
set -o pipefail
O=gpurun_out
for q in ${QUEUES:-4 16}; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u tools/c3_probe.py 16384 > $O/hwq_c3_$q.json 2> $O/hwq_c3_$q.err || { tail -5 $O/hwq_c3_$q.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hwq_c3_$q.json')); g=d['go_wiring']
print('q=$q c3', round(d['messages_per_s']/1e6,1), 'go', round(g['messages_per_s']/1e6,1), {k: round(v['messages_per_s']/1e6,1) for k,v in g['coalesced'].items()})"
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 > $O/hwq_bench_$q.json 2> $O/hwq_bench_$q.err || { tail -5 $O/hwq_bench_$q.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/hwq_bench_$q.json'))
print('q=$q c2', round(d['value']/1e6,1), 'auth p50', round(d['p50_batch_latency_ms'],3), 'single', round(d['single_calls']['p50_latency_us'],1), 'conc', {k: round(v['calls_per_s']/1e6,1) for k,v in d['concurrent_batches'].items() if isinstance(v, dict)})"
done
