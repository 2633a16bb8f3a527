#!/bin/bash
# Round 4 session 6: every GPU test (host graph lookups changed), the storm bench, kernel stats
# of the C4 edge-cut at P = 1 and 8 (in one process), and the frontier stall counters at the
# merged distinct-batch kernel with the locality layout (profiles/r04_pmc_frontier_layout.txt).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s6
mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));c=d['config'];print('storm', round(d['value']), round(d['ms_per_step'],2), {k: round(v,3) for k,v in c['stage_ms_mean'].items()}, c['reseed_per_tick'])"
for P in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard_p$P -o run -- python3 bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline > $OUT/shard_p$P.json 2> $OUT/shard_p$P.err
  echo "shard P=$P prof ok"
done
TAG=r04s6/pmc BENCH_ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-dropin --dense-steps 0" bash scripts/pmc_frontier.sh
python scripts/pmc_summary.py gpurun_out/r04s6/pmc > $OUT/pmc_summary.txt 2>&1 || true
head -40 $OUT/pmc_summary.txt
