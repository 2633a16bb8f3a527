#!/bin/bash
# A/B several libegraph.so variants (VARIANTS="name=path ..."; "base" = the default build) on
# the bench, interleaved REPS times.  One GPU call; every bench run under its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abm}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  for nv in ${VARIANTS:-base=}; do
    n=${nv%%=*}; p=${nv#*=}
    if [ -n "$p" ]; then export EGRAPH_LIB=$PWD/$p; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/$n.$r.json 2> $OUT/$n.$r.err
    python -c "import json;d=json.load(open('$OUT/$n.$r.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$n rep $r', round(d['value']), round(d['ms_per_step'],4), 'launch', round(r['avg_launch_ms'],4), 'members', w.get('members'), 'ovf', w.get('overflowed'))"
  done
done
