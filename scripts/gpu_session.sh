#!/bin/bash
# One GPU call: gpu tests + default bench, then member distribution and an optional library A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-session}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
if [ -n "$MEMBERS" ]; then
  timeout -k 10 200 python -u scripts/frontier_members.py C3 > $OUT/members_c3.json 2>&1
  cat $OUT/members_c3.json | tail -1
fi
if [ -n "$ALT" ]; then TAG=${TAG:-session}/ab bash scripts/ab_lib.sh; fi
