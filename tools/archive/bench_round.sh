set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt_$TAG -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peak-run --no-adversarial --c3-requests 0 --no-extra-lines > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?
[ $rc -eq 0 ] && python3 tools/trace_summary.py gpurun_out/prof_kt_$TAG/kt_kernel_trace.csv > gpurun_out/kt_summary_$TAG.json
echo rc=$rc
exit $rc
