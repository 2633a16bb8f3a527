#!/bin/bash
# Round 4 session 40: the narrow table at seven workgroups per CU (exp_n7: a 2^14-bit filter,
# 22 KB of LDS, 72 VGPRs with 14 spilled) vs the committed tree (six per CU): frontier + config
# parity with exp_n7, then the C3 headline launch at --steps 20, interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s40
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$L/exp_n7/libegraph.so timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_n7.log 2>&1
echo "n7 parity: $(tail -1 $OUT/pytest_n7.log)" | tee -a $OUT/ab.txt
for i in 1 2; do
  for v in base n7; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c3_$v$i.json'));r=d['roofline'];print('C3 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
