#!/bin/bash
# A/B of variant libraries on C4 (wide-first) and C3: parity tests first, then the benches.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abw}
mkdir -p $OUT
L=kubernetes-aiops-evidence-graph_amd/lib
for v in default ${ALTS}; do
  if [ $v = default ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/$v/libegraph.so; fi
  timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  echo "$v tests: $(tail -n 1 $OUT/pytest_$v.log)"
done
for rep in 1 2; do
  for v in default ${ALTS}; do
    if [ $v = default ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/$v/libegraph.so; fi
    for C in C4 C3; do
      timeout -k 10 300 python bench.py --config $C --no-cpu-baseline --no-dropin --dense-steps 0 --steps 200 > $OUT/${v}_$C.json 2> $OUT/${v}_$C.err
      python -c "import json;d=json.load(open('$OUT/${v}_$C.json'));print('$v $C', round(d['value']), round(d['ms_per_step'],4))"
    done
  done
done
