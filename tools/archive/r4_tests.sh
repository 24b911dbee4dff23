#!/bin/bash
# GPU tests only (selected with -k when given), each step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
else
  timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
fi
rc=$?
tail -15 gpurun_out/pytest_$TAG.log
exit $rc
