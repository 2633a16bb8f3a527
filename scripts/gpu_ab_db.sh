#!/bin/bash
# FR_DBUF narrow frontier: parity tests against the variant library, then an interleaved A/B.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-abdb} LIBS="default ${ALTS:-exp_db1536}" REPS="1 2" STEPS=200 \
  TESTS="tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_frontier_scale_gpu.py" \
  bash scripts/ab_multi.sh
