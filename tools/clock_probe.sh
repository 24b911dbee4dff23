#!/bin/bash
# Clock / power under sustained verify load: a long bench run (2,000 steps
# of 1M verifies) in the background while amd-smi samples the GPU's power
# and clocks every ~0.3 s; then the same for synchronized single batches.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2000 --warmup 5 --latency-reps 3 --no-cpu-baseline --no-peak-run \
  > gpurun_out/clk/bench_long.json 2> gpurun_out/clk/bench_long.err &
pid=$!
for k in $(seq 1 200); do
  kill -0 $pid 2>/dev/null || break
  { echo "T $(date +%s.%N)"; timeout 5 amd-smi metric -g 0 -p -c 2>&1; timeout 5 rocm-smi -d 0 --showpower --showclocks 2>&1; } >> gpurun_out/clk/samples.txt
  sleep 0.3
done
wait $pid
echo "bench rc=$?"
python3 -c "import json;d=json.load(open('gpurun_out/clk/bench_long.json'));print('long value %.1fM ms/step %.4f k_verify %.4f'%(d['value']/1e6,d['ms_per_step'],d['kernel_ms']['k_verify']))"
