#!/bin/bash
# Round 4 session 23: the mid table's light-row limit (FR_LMAX_MID 12 = exp_hpf, 16/20/24/32 =
# exp_ml*): C4 parity with each, then C4 (mid-first) at --steps 20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s23
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
for v in ml16 ml24 ml32; do
  EGRAPH_LIB=$L/exp_$v/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k c4_frontier > $OUT/pytest_$v.log 2>&1
  echo "$v C4 parity: $(tail -1 $OUT/pytest_$v.log)" | tee -a $OUT/ab.txt
done
for i in 1 2; do
  for v in hpf ml16 ml20 ml24 ml32; do
    export EGRAPH_LIB=$L/exp_$v/libegraph.so
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];w=d['frontier_work'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'], w['overflowed'])" | tee -a $OUT/ab.txt
  done
done
