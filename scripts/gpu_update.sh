#!/bin/bash
# GPU tests of the incremental snapshot update (and the alert front end).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-update}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_update_gpu.py} -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -80 $OUT/pytest.log; exit 1; }
tail -15 $OUT/pytest.log
