#!/bin/bash
# Round 4 session 32: the mid table's light-row limit with light-row tails (head 8): FR_LMAX 24
# (exp_ml24) and 32 (exp_ml32) against the committed 16 -- C4 parity with each, then C4
# (mid-first) at --steps 20, interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s32
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
for v in ml24 ml32; do
  EGRAPH_LIB=$L/exp_$v/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k c4_frontier > $OUT/pytest_$v.log 2>&1
  echo "$v C4 parity: $(tail -1 $OUT/pytest_$v.log)" | tee -a $OUT/ab.txt
done
for i in 1 2; do
  for v in base ml24 ml32; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'], d['frontier_work']['overflowed'])" | tee -a $OUT/ab.txt
  done
done
