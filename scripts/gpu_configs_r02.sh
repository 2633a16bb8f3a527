#!/bin/bash
# C2 and C4 frontier benches at the current defaults (and A/B libraries in LIBS).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-cfg}
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
for v in ${LIBS:-default}; do
  if [ $v = default ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/$v/libegraph.so; fi
  for C in ${CONFIGS:-C2 C4}; do
    timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-dropin --dense-steps 0 --steps 100 > $OUT/${v}_$C.json 2> $OUT/${v}_$C.err
    python -c "import json;d=json.load(open('$OUT/${v}_$C.json'));w=d.get('frontier_work',{});print('$v $C', round(d['value']), round(d['ms_per_step'],4), 'members', w.get('members'), 'ovf', w.get('overflowed'), 'global', w.get('global_columns'))"
  done
done
