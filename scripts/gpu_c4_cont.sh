#!/bin/bash
# C4 replicated frontier: the mid-table continuation A/B (regions sized by adapt() vs
# EGRAPH_FRONTIER_CONTINUATION=0: the mid table + the serial wide retry), after the C4 tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-c4cont}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -k "c4_launch_m20 or c4_frontier_b256" > $OUT/pytest.log 2>&1
echo "tests: $(tail -1 $OUT/pytest.log)"
for r in 1 2; do
for alt in cont off; do
  if [ $alt = off ]; then export EGRAPH_FRONTIER_CONTINUATION=0; fi
  timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_${alt}_$r.json 2> $OUT/c4_${alt}_$r.err
  python -c "import json;d=json.load(open('$OUT/c4_${alt}_$r.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$alt', round(d['value']), round(d['ms_per_step'],4), 'launch', round(r['avg_launch_ms'],4), d['config']['first_table'], 'ovf', w.get('overflowed'), 'cont', w.get('continued'), 'global', w.get('global_columns'))"
  unset EGRAPH_FRONTIER_CONTINUATION
done
done
