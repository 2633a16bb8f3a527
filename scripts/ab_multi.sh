#!/bin/bash
# A/B several libegraph.so builds on the bench (EGRAPH_LIB per variant; "default" = lib/).
# LIBS: space-separated variant names (default exp_old ...); PIPES: pipeline depths;
# TESTS: pytest node ids run against every variant first (parity before speed).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abm}
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
for v in ${LIBS:-default}; do
  if [ $v = default ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/$v/libegraph.so; fi
  if [ -n "$TESTS" ]; then
    timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
    echo "$v tests: $(tail -n 1 $OUT/pytest_$v.log)"
  fi
done
for rep in ${REPS:-1}; do
for P in ${PIPES:-3}; do
  for v in ${LIBS:-default}; do
    if [ $v = default ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/$v/libegraph.so; fi
    timeout -k 10 200 python bench.py --pipeline $P --no-cpu-baseline --no-dropin --dense-steps 0 --steps ${STEPS:-200} ${BENCH_ARGS:-} > $OUT/${v}_P$P.json 2> $OUT/${v}_P$P.err
    python -c "import json;d=json.load(open('$OUT/${v}_P$P.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v P=$P', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), 'members', w.get('members'), 'ovf', w.get('overflowed'))"
  done
done
done
