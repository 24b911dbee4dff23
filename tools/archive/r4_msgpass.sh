#!/bin/bash
# Message-layer pass work (round 4): the GPU tests it touches, the single-pass
# probe (one-wait and two-wait forms), then the hardware-queue A/B.
set -o pipefail
O=gpurun_out
TAG=${1:-mp}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_msgdev.py tests/test_gpu_check_coalesce.py tests/test_gpu_keys_late.py > $O/pytest_mp_$TAG.log 2>&1 || { tail -40 $O/pytest_mp_$TAG.log; exit 1; }
tail -2 $O/pytest_mp_$TAG.log
timeout -k 10 200 python -u tools/msg_pass_probe.py 40 > $O/mp_onewait_$TAG.json 2> $O/mp_onewait_$TAG.err || { tail -5 $O/mp_onewait_$TAG.err; exit 1; }
MBFT_MSG_ONE_WAIT=0 timeout -k 10 200 python -u tools/msg_pass_probe.py 40 > $O/mp_twowait_$TAG.json 2> $O/mp_twowait_$TAG.err || { tail -5 $O/mp_twowait_$TAG.err; exit 1; }
cat $O/mp_onewait_$TAG.json $O/mp_twowait_$TAG.json
if [ "${HWQ:-1}" = 1 ]; then QUEUES="4 16" bash tools/hwq_ab.sh; fi
