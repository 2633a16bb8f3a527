#!/bin/bash
# Round 4 session 8: the fixed-slot exchange as count (lane-per-row work map) + scan + emit with
# the per-peer counts taken from the scan (partition tests, C4 at P = 1/2/4/8, kernel stats at
# P = 8), then an A/B of the dense hop with XCD-contiguous block runs ($ALT, -DEGR_HOP_XCD_REMAP=1):
# dense-engine step time and the hop kernel's L2->HBM read requests per launch.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s8
mkdir -p $OUT
TAG=r04s8/shard bash scripts/gpu_shard.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard_p8 -o run -- python3 bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/shard_p8.json 2> $OUT/shard_p8.err
echo "shard P=8 prof ok"
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04s8/shard_p8/run_kernel_stats.csv")))
for r in rows[:10]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
ALT=kubernetes-aiops-evidence-graph_amd/lib/exp_xcd/libegraph.so
DA="--steps 2 --warmup 1 --dense-steps 5 --no-cpu-baseline --no-dropin"
for i in 1 2; do
  for v in base alt; do
    if [ $v = alt ]; then export EGRAPH_LIB=$PWD/$ALT; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py $DA > $OUT/dense_$v$i.json 2> $OUT/dense_$v$i.err
    python -c "import json;d=json.load(open('$OUT/dense_$v$i.json'))['dense_engine'];r=d['roofline'];print('dense $v $i', round(d['ms_per_step'],3), 'hop ms', round(r['avg_launch_ms'],3), 'frac', round(r['frac'],3))" | tee -a $OUT/ab_xcd.txt
  done
done
for v in base alt; do
  if [ $v = alt ]; then export EGRAPH_LIB=$PWD/$ALT; else unset EGRAPH_LIB; fi
  timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d $OUT/rdreq_$v -o rdreq -- python3 bench.py $DA > $OUT/rdreq_$v.log 2>&1
  echo "rdreq $v ok"
  python scripts/pmc_summary.py $OUT/rdreq_$v "hop_kernel<32, false>" | tee -a $OUT/ab_xcd.txt
done
unset EGRAPH_LIB
