#!/bin/bash
# Round 6: a chosen set of GPU tests ($@), one pytest process, its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${R6TAG:-r6t}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
