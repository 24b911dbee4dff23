#!/bin/bash
# Same-box A/B of the C3 message layer (tools/c3_probe.py with the stage
# trace) between the in-tree library and minbft_amd/libminbft_amd_<TAG>.so.
#   bash tools/c3_ab.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c3ab
for rep in 1 2 3; do
  for tag in new "$1"; do
    if [ "$tag" = new ]; then L=""; else L="$PWD/minbft_amd/libminbft_amd_$tag.so"; fi
    MBFT_LIB_PATH=$L MBFT_STAGE_TRACE=1 timeout -k 10 300 python tools/c3_probe.py > gpurun_out/c3ab/${tag}_$rep.json 2> gpurun_out/c3ab/${tag}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c3ab/${tag}_$rep.json'));print('$tag rep $rep %.2f M msgs/s %.1f ms'%(d['messages_per_s']/1e6, d['ms']))"
    grep "mbft validate" gpurun_out/c3ab/${tag}_$rep.err | tail -1
  done
done
