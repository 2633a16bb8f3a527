#!/bin/bash
# Round 4 session 27: light-row tails spread over the wave (FR_HEAD entries per row in-lane, the
# rest one entry per lane, chains continued from the pair scratch): exp_h4m8 (narrow head 4,
# mid 8), exp_h4m4, exp_h0m8 (narrow unchanged) vs the committed tree; parity suites with
# exp_h4m8 (C4 parity with exp_h4m4), then the C3 headline launch and C4 (mid-first) at --steps 20;
# exp_m3k = exp_h4m8 with a 3072-slot mid table (2304 members, 2^14-bit filter; 52 KB, still 3 per CU);
# exp_dq = exp_h4m8 with the wide retry drained through a work queue instead of a static stride.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s27
mkdir -p $OUT
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$L/exp_h4m8/libegraph.so timeout -k 10 500 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_h4m8.log 2>&1
echo "h4m8 tests ok"; tail -1 $OUT/pytest_h4m8.log
EGRAPH_LIB=$L/exp_h4m4/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k c4_frontier > $OUT/pytest_h4m4.log 2>&1
echo "h4m4 C4 ok"; tail -1 $OUT/pytest_h4m4.log
EGRAPH_LIB=$L/exp_m3k/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k c4_frontier > $OUT/pytest_m3k.log 2>&1
echo "m3k C4 ok"; tail -1 $OUT/pytest_m3k.log
EGRAPH_LIB=$L/exp_dq/libegraph.so timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_frontier_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c4_frontier or retry or overflow or wide" > $OUT/pytest_dq.log 2>&1
echo "dq ok"; tail -1 $OUT/pytest_dq.log
for i in 1 2; do
  for v in base h4m8 h4m4 h0m8 m3k dq; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    if [ $v != h4m4 ] && [ $v != m3k ] && [ $v != dq ]; then
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c3_$v$i.json'));r=d['roofline'];print('C3 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
    fi
    if [ $v != h0m8 ]; then
    timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$v$i.json 2> $OUT/c4_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c4_$v$i.json'));r=d['roofline'];print('C4 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'], d['frontier_work']['overflowed'])" | tee -a $OUT/ab.txt
    fi
  done
done
