#!/bin/bash
# GPU tests, then the bench with and without the pruned last pull (EGRAPH_FRONTIER_NO_PRUNE).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-prune}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
for v in prune noprune prune; do
  if [ $v = noprune ]; then export EGRAPH_FRONTIER_NO_PRUNE=1; else unset EGRAPH_FRONTIER_NO_PRUNE; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 --steps 50 > $OUT/$v.json 2> $OUT/$v.err
  python -c "import json;d=json.load(open('$OUT/$v.json'));r=d['roofline'];w=d['frontier_work'];print('$v', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), w['pull_entries'])"
done
