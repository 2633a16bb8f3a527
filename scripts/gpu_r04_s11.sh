#!/bin/bash
# Round 4 session 11: partitioned hops write each (row, tile)'s non-zero COUNT (a seed add marks
# the tile unknown), so the fixed-slot pack's count pass sums bytes instead of re-reading the
# scores: every GPU test, C4 at P = 1/2/4/8 (scripts/gpu_shard.sh), kernel stats at P = 8.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s11
mkdir -p $OUT
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -1 $OUT/pytest_gpu.log
TAG=r04s11/shard bash scripts/gpu_shard.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard_p8 -o run -- python3 bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/shard_p8.json 2> $OUT/shard_p8.err
echo "shard P=8 prof ok"
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04s11/shard_p8/run_kernel_stats.csv")))
for r in rows[:12]:
    print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
