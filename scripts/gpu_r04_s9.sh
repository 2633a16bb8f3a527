#!/bin/bash
# Round 4 session 9: edge-cut with the strided work-map exchange kernels and the reach chain on
# its own stream: partition tests, C4 at P = 1/2/4/8 (scripts/gpu_shard.sh), P = 8 without the
# overlap (A/B of the in-process step), kernel stats at P = 8, C4 through the replicated frontier.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s9
mkdir -p $OUT
TAG=r04s9/shard bash scripts/gpu_shard.sh
for ov in "" "--no-overlap"; do
  timeout -k 10 200 python -u bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline $ov > $OUT/c4_p8$ov.json 2> $OUT/c4_p8$ov.err
  python -c "import json;d=json.load(open('$OUT/c4_p8$ov.json'));c=d['config'];print('P=8 $ov', round(d['ms_per_step'],2), 'ms in-process; serial', [round(x,2) for x in c['partition_compute_ms']], 'critical', [round(x,2) for x in c['partition_critical_ms']], 'projected', round(c['projected_ms_per_gpu'],2), 'serial projected', round(c['projected_serial_ms_per_gpu'],2), 'link B/step', c['link_bytes_per_step_max_rank'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard_p8 -o run -- python3 bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/shard_p8.json 2> $OUT/shard_p8.err
echo "shard P=8 prof ok"
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04s9/shard_p8/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
# C4 through the replicated frontier (distinct batches, merged launch, wide-first after adapt)
timeout -k 10 300 python -u bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_frontier.json 2> $OUT/c4_frontier.err
python -c "import json;d=json.load(open('$OUT/c4_frontier.json'));print('C4 frontier', round(d['value']), round(d['ms_per_step'],4), d.get('frontier_work'))"
