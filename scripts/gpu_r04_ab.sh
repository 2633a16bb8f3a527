#!/bin/bash
# Round 4 session B: every GPU test on the tree (storm SeedStore, open-addressing host graph,
# distinct-batch bench), then an interleaved A/B of a variant libegraph.so ($ALT) against the
# default build at the driver's settings, the variant's frontier parity tests, and the storm
# bench.  Produces profiles/r04_ab_*.txt, r04_storm_*.json.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r04ab}
mkdir -p $OUT
ALT=${ALT:-kubernetes-aiops-evidence-graph_amd/lib/exp_spec/libegraph.so}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
fi
EGRAPH_LIB=$PWD/$ALT timeout -k 10 300 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "frontier or c3 or merged" > $OUT/pytest_alt.log 2>&1
echo "alt tests ok"; tail -1 $OUT/pytest_alt.log
for i in 1 2 3; do
  for v in base alt; do
    if [ $v = alt ]; then export EGRAPH_LIB=$PWD/$ALT; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), 'members', w.get('members'), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
if [ -z "$SKIP_STORM" ]; then
  timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
  python -c "import json;d=json.load(open('$OUT/storm.json'));c=d['config'];print('storm', round(d['value']), round(d['ms_per_step'],2), c['stage_ms_mean'], c['reseed_per_tick'])"
fi
