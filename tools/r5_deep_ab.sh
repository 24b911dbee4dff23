#!/bin/bash
# Two-deep vs one-deep comb gathers (kernels.hip comb_verify_fast2), same box:
# (builds: bash tools/ab_build_def.sh two "-DMBFT_TWO_DEEP_GATHER"; the default build is one-deep)
# parity tests on the new kernel, then k_verify isolated (tools/step_timing.py)
# at 3 and 1 waves / SIMD, and the C2 steady state (bench.py, short), each lib
# twice in alternation.  Each GPU step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/deep
export TMPDIR=/tmp
O=gpurun_out/deep
if [ "${1:-}" != "notest" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "bench_config or parity or c1 or golden or field" --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for rep in 1 2; do
  for lib in two one; do
    if [ $lib = one ]; then L=minbft_amd/libminbft_amd.so; else L=minbft_amd/libminbft_amd_two.so; fi
    MBFT_LIB_PATH=$L timeout -k 10 240 python -u tools/step_timing.py > $O/iso3_${lib}_$rep.json 2>>$O/err.log || exit 1
    MBFT_VERIFY_BPC=1 MBFT_LIB_PATH=$L timeout -k 10 240 python -u tools/step_timing.py > $O/iso1_${lib}_$rep.json 2>>$O/err.log || exit 1
    MBFT_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-adversarial --c3-requests 0 --no-extra-lines --no-cpu-baseline > $O/bench_${lib}_$rep.json 2>>$O/err.log || exit 1
  done
done
python3 - <<'PY'
import json, glob
for lib in ("two", "one"):
    for rep in (1, 2):
        i3 = json.load(open(f"gpurun_out/deep/iso3_{lib}_{rep}.json"))
        i1 = json.load(open(f"gpurun_out/deep/iso1_{lib}_{rep}.json"))
        b = json.load(open(f"gpurun_out/deep/bench_{lib}_{rep}.json"))
        print(lib, rep, "iso3 %.3f ms  iso1 %.3f ms  C2 %.1f M/s  ms/step %.4f  frac %.3f" % (
            i3["k_verify_ms"], i1["k_verify_ms"], b["value"] / 1e6, b["ms_per_step"], b["roofline"]["frac"]))
PY
