#!/bin/bash
# Round 4 session 15: the narrow table's member limit (LLIMIT 1152 of 1536 slots) against 1280 /
# 1344 (fewer columns overflow to the wide retry at a higher load): parity tests of both variants,
# interleaved A/B with the overflow counts.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s15
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
for v in ll1280; do
  EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "frontier or c3 or merged or C4" > $OUT/pytest_$v.log 2>&1
  echo "tests $v ok"; tail -1 $OUT/pytest_$v.log
done
BA="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
for i in 1 2; do
  for v in base ll1280 ll1344; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 200 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
