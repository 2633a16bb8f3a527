#!/bin/bash
# Fallback-at-scale tests, the GPU suite, then the bench with / without the wide-table retry
# and without pruning.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-retry}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_frontier_scale_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_scale.log 2>&1
echo "scale tests ok"; tail -1 $OUT/pytest_scale.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -1 $OUT/pytest_gpu.log
for v in retry noretry retry noretry noprune; do
  unset EGRAPH_FRONTIER_WIDE_RETRY EGRAPH_FRONTIER_NO_PRUNE
  if [ $v = retry ]; then export EGRAPH_FRONTIER_WIDE_RETRY=1; fi
  if [ $v = noprune ]; then export EGRAPH_FRONTIER_NO_PRUNE=1; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 --steps 50 > $OUT/$v.json 2> $OUT/$v.err
  python -c "import json;d=json.load(open('$OUT/$v.json'));w=d['frontier_work'];print('$v', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), w['overflowed'], w['corrupt_keys'])"
done
