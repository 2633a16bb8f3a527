#!/bin/bash
# Round 4 session 19: C4 replicated frontier, mid-first ($EGRAPH_FRONTIER_MID=1), probe width
# A/B: buckets read per lockstep probe round in the mid (m2, m3) and wide (w2) geometries.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s19
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
export EGRAPH_FRONTIER_MID=1
EGRAPH_LIB=$PWD/$L/exp_m2/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_frontier_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c4 or C4 or overflow or wide" > $OUT/pytest_m2.log 2>&1
echo "m2 tests ok"; tail -1 $OUT/pytest_m2.log
BA="--config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
for i in 1 2; do
  for v in base m2 m3 m2w2; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'), 'glob', w.get('global_columns'))" | tee -a $OUT/ab.txt
  done
done
