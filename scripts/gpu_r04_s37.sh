#!/bin/bash
# Round 4 session 37: the mid table with one LDS score buffer (exp_md0: FR_DBUF 0, pull results
# by member index in HBM + a copy phase) -- 39 KB, four workgroups per CU instead of three --
# vs the committed tree: frontier + config parity with exp_md0, then C4 (mid-first) at --steps 20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s37
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$L/exp_md0/libegraph.so timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_md0.log 2>&1
echo "md0 parity: $(tail -1 $OUT/pytest_md0.log)" | tee -a $OUT/ab.txt
for i in 1 2; do
  for v in base md0; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])" | tee -a $OUT/ab.txt
  done
done
