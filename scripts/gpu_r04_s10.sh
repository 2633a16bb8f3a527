#!/bin/bash
# Round 4 session 10: the frontier's heavy split (costliest-predicted columns on the wide grid on a
# second stream from the start) -- parity tests, interleaved A/B against $EGRAPH_FRONTIER_HEAVY=0,
# kernel stats -- and the edge-cut with the weight-balanced partition (C4 at P = 1/2/4/8).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s10
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_layout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
BA="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
for i in 1 2; do
  for v in on off; do
    if [ $v = off ]; then export EGRAPH_FRONTIER_HEAVY=0; else unset EGRAPH_FRONTIER_HEAVY; fi
    timeout -k 10 200 python bench.py $BA > $OUT/heavy_$v$i.json 2> $OUT/heavy_$v$i.err
    python -c "import json;d=json.load(open('$OUT/heavy_$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('heavy $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab_heavy.txt
  done
done
unset EGRAPH_FRONTIER_HEAVY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py $BA > $OUT/prof.log 2>&1
echo "prof ok"
head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-160
TAG=r04s10/shard bash scripts/gpu_shard.sh
