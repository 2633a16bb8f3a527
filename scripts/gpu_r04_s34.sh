#!/bin/bash
# Round 4 session 34: geometry knobs after the light-row tails -- narrow with branch-free probes
# (exp_nsel), narrow head 8 (exp_nh8), mid head 12 (exp_mh12) vs the committed tree: frontier
# parity suites with each, then the C3 headline launch (nsel, nh8) / C4 (mh12) at --steps 20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s34
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
for v in nsel nh8 mh12; do
  EGRAPH_LIB=$L/exp_$v/libegraph.so timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
  echo "$v parity: $(tail -1 $OUT/pytest_$v.log)" | tee -a $OUT/ab.txt
done
for i in 1 2; do
  for v in base nsel nh8; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c3_$v$i.json'));r=d['roofline'];print('C3 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
  for v in base mh12; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])" | tee -a $OUT/ab.txt
  done
done
