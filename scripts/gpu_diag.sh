#!/bin/bash
# Frontier tests, then the bench pruned and unpruned, printing the work counters (incl. the
# corrupt-key guard).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-diag}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_frontier_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_frontier.log 2>&1
echo "frontier tests ok"; tail -1 $OUT/pytest_frontier.log
for v in prune noprune; do
  if [ $v = noprune ]; then export EGRAPH_FRONTIER_NO_PRUNE=1; else unset EGRAPH_FRONTIER_NO_PRUNE; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 --steps 20 ${BENCH_ARGS:-} > $OUT/$v.json 2> $OUT/$v.err
  python -c "import json;d=json.load(open('$OUT/$v.json'));print('$v', round(d['value']), round(d['ms_per_step'],4), d['frontier_work'])"
done
