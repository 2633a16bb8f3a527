#!/bin/bash
# Round 4 session 5: the many-block device launch order (tests, bench, kernel stats), an A/B of a
# 6-waves-per-SIMD narrow frontier ($ALT: no second LDS score buffer, 80 VGPRs) against the
# default build, the storm bench (deferred deallocation, pending-index runs), the drop-in host
# profile and the seed_keys thread-scaling microbenchmark on the box's CPU share.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s5
mkdir -p $OUT
bash scripts/gpu_r04_order.sh
ALT=kubernetes-aiops-evidence-graph_amd/lib/exp_w6/libegraph.so
EGRAPH_LIB=$PWD/$ALT timeout -k 10 300 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "frontier or c3 or merged" > $OUT/pytest_alt.log 2>&1
echo "alt tests ok"; tail -1 $OUT/pytest_alt.log
for i in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export EGRAPH_LIB=$PWD/$ALT; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), 'members', w.get('members'), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));c=d['config'];print('storm', round(d['value']), round(d['ms_per_step'],2), c['stage_ms_mean'], c['reseed_per_tick'])"
timeout -k 10 300 python -u scripts/prof_dropin.py > $OUT/prof_dropin.txt 2> $OUT/prof_dropin.err
echo "prof_dropin ok"; grep -m3 "concurrent ms\|generate_hypotheses x\|dropin_graph" $OUT/prof_dropin.txt
timeout -k 10 200 python -u scripts/cpu_seedkeys.py > $OUT/cpu_seedkeys.txt 2>&1
cat $OUT/cpu_seedkeys.txt
