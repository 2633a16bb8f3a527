#!/bin/bash
# Round 4 experiment: the same C3 workload (20 distinct incident sets) MERGEd in the natural
# order vs in egraph.graph.locality_order (EGRAPH_BENCH_HUB_ORDER=1), interleaved three times at
# the driver's settings, plus TCC_EA0_RDREQ of both.  Produces profiles/r04_ab_hub_order.txt.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r04hub}
mkdir -p $OUT
for i in 1 2 3; do
  for v in base hub; do
    if [ $v = hub ]; then export EGRAPH_BENCH_HUB_ORDER=1; else unset EGRAPH_BENCH_HUB_ORDER; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];w=d.get('frontier_work',{});print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3), 'members', w.get('members'), 'pulls', w.get('pull_entries'), 'ovf', w.get('overflowed'))" | tee -a $OUT/ab.txt
  done
done
P="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
unset EGRAPH_BENCH_HUB_ORDER
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum --output-format csv -d $OUT/rdreq_base -o rdreq -- python3 bench.py $P > $OUT/rdreq_base.log 2>&1
echo "rdreq base ok"
export EGRAPH_BENCH_HUB_ORDER=1
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum --output-format csv -d $OUT/rdreq_hub -o rdreq -- python3 bench.py $P > $OUT/rdreq_hub.log 2>&1
echo "rdreq hub ok"
python scripts/pmc_summary.py $OUT/rdreq_base frontier_lds_kernel
python scripts/pmc_summary.py $OUT/rdreq_hub frontier_lds_kernel
