#!/bin/bash
# Round 6: the driver's bench command with the default build, then with an
# A/B build ($ABLIB, lighter run), alternated: default, AB, default.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6h}
mkdir -p $O
X="--no-adversarial --c3-requests 0"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --detail-out $O/detail_a1.json > $O/bench_a1.json 2> $O/bench_a1.err || { tail -30 $O/bench_a1.err; exit 1; }
MBFT_LIB_PATH=$ABLIB timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 $X --detail-out $O/detail_b1.json > $O/bench_b1.json 2> $O/bench_b1.err || { tail -30 $O/bench_b1.err; exit 1; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 $X --detail-out $O/detail_a2.json > $O/bench_a2.json 2> $O/bench_a2.err || { tail -30 $O/bench_a2.err; exit 1; }
echo "[r6_bench_ab] done"
