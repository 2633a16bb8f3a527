#!/bin/bash
# Round 4: the frontier's locality layout (csrc/layout.hip).  Parity tests (layout vs canonical
# vs oracle, after updates, partition-local snapshots, and the frontier / config tests with the
# layout on), then an interleaved A/B of the layout against EGRAPH_FRONTIER_LAYOUT=0 at the
# driver's settings, and the bytes past L2 with the layout.  Produces profiles/r04_ab_layout.txt.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r04lay}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread > $OUT/pytest_rccl.log 2>&1 && echo "rccl test ok" || { echo "rccl test FAILED"; tail -30 $OUT/pytest_rccl.log; }
timeout -k 10 400 python -u -m pytest tests/test_layout_gpu.py tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_storm_gpu.py tests/test_frontier_scale_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
for i in 1 2 3; do
  for v in off on; do
    if [ $v = off ]; then export EGRAPH_FRONTIER_LAYOUT=0; else unset EGRAPH_FRONTIER_LAYOUT; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), 'members', w.get('members'), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_FRONTIER_LAYOUT
P="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum --output-format csv -d $OUT/rdreq -o rdreq -- python3 bench.py $P > $OUT/rdreq.log 2>&1
echo "rdreq ok"
python scripts/pmc_summary.py $OUT/rdreq frontier_lds_kernel
