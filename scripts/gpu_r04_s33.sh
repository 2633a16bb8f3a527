#!/bin/bash
# Round 4 session 33: the wide table with the mid table's light-row treatment (exp_w2: hub chains
# through the LDS scratch, light-row tails with head 8, limit 16, a 2^15-bit filter to stay at
# two 80-KB workgroups per CU) vs the committed tree: frontier parity suites (incl. the
# fallback-scale tests) with exp_w2, then C4 (mid-first: its overflows re-run in the wide table)
# and the C3 headline launch at --steps 20, interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s33
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$L/exp_w2/libegraph.so timeout -k 10 500 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_frontier_scale_gpu.py tests/test_layout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_w2.log 2>&1
echo "w2 parity: $(tail -1 $OUT/pytest_w2.log)" | tee -a $OUT/ab.txt
for i in 1 2; do
  for v in base w2; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'], d['frontier_work']['overflowed'])" | tee -a $OUT/ab.txt
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c3_$v$i.json'));r=d['roofline'];print('C3 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
