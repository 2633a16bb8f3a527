#!/bin/bash
# A/B a variant libegraph.so (EGRAPH_LIB=$ALT) against the default build on the bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
ALT=${ALT:-kubernetes-aiops-evidence-graph_amd/lib/exp/libegraph.so}
if [ -n "$TESTS" ]; then
  EGRAPH_LIB=$PWD/$ALT timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_alt.log 2>&1
  echo "alt tests ok"; tail -1 $OUT/pytest_alt.log
fi
for P in ${PIPES:-1 2}; do
  for v in base alt; do
    if [ $v = alt ]; then export EGRAPH_LIB=$PWD/$ALT; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py --pipeline $P --no-cpu-baseline --no-dropin --dense-steps 0 --steps 50 ${BENCH_ARGS:-} > $OUT/$v$P.json 2> $OUT/$v$P.err
    python -c "import json;d=json.load(open('$OUT/$v$P.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v P=$P', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), r.get('traffic'), 'members', w.get('members'), 'ovf', w.get('overflowed'))"
  done
done
