#!/bin/bash
# Copy / kernel timeline of the authenticator level on the GPU box: the
# probe (tools/auth_level_probe.py, 1M C2 calls, 3 reps) under rocprofv3
# --kernel-trace --memory-copy-trace, once per form (host decode over an
# item array; GPU decode over page-locked flat buffers), then
# tools/copy_timeline.py over the last batch.  Output in gpurun_out/.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for form in ${MBFT_TL_FORMS:-items pinned}; do
  MBFT_PROBE_FORM=$form MBFT_STAGE_TRACE=1 timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace \
    --output-format csv -d gpurun_out/tl_$form -o tl -- python3 tools/auth_level_probe.py 1048576 3 \
    > gpurun_out/tl_$form.json 2> gpurun_out/tl_$form.err || exit 1
  python3 tools/copy_timeline.py gpurun_out/tl_$form/tl 8 > gpurun_out/tl_$form.txt || exit 1
done
