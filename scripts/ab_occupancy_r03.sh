#!/bin/bash
# Round 3 A/B: the narrow frontier table at 1280 slots (six workgroups per CU, 80 VGPRs with a
# few spills) against the shipped 1536 (five per CU), merged schedule, one box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab_occ}
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$PWD/$L/exp_n6/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "merged" > $OUT/pytest_n6.log 2>&1
echo "n6 tests ok"; tail -1 $OUT/pytest_n6.log
for rep in 1 2; do
  for v in base n6 n6b; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 --steps 240 > $OUT/$v$rep.json 2> $OUT/$v$rep.err
    python -c "import json;d=json.load(open('$OUT/$v$rep.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v rep $rep', round(d['ms_per_step'],4), round(d['value']/1e6,2), 'launch', round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'), 'glob', w.get('global_columns'))"
  done
done
