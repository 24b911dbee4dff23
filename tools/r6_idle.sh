#!/bin/bash
# Round 6: the idle batch's s^-1 form (bench p50_batch_latency_device_ms),
# alternated on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6idle}
mkdir -p $O
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python3 tools/idle_batch_probe.py > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; return 1; }; echo "$tag $(cat $O/$tag.json)"; }
run block8 MBFT_X=1 && run block4 MBFT_NINV_PER=4 && run wave16 MBFT_NINV_FORM=wave MBFT_NINV_PER=16 && run wave8 MBFT_NINV_FORM=wave MBFT_NINV_PER=8 && run block8b MBFT_X=1 && run wave16b MBFT_NINV_FORM=wave MBFT_NINV_PER=16 || exit 1
echo "[r6_idle] done"
