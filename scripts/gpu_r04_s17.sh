#!/bin/bash
# Round 4 session 17: C4 through the replicated frontier with a 2.8k-slot, 256-thread first
# attempt (fr_mid, three workgroups per CU) instead of wide-first ($EGRAPH_FRONTIER_MID=1):
# the C4 frontier parity test with it, then interleaved C4 benches with / without.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s17
mkdir -p $OUT
EGRAPH_FRONTIER_MID=1 timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c4_frontier" > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
BA="--config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
for i in 1 2; do
  for v in mid wide; do
    if [ $v = mid ]; then export EGRAPH_FRONTIER_MID=1; else unset EGRAPH_FRONTIER_MID; fi
    timeout -k 10 300 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'), 'glob', w.get('global_columns'))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_FRONTIER_MID
