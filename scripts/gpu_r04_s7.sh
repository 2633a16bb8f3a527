#!/bin/bash
# Round 4 session 7: the one-launch fixed-slot pack (sx_emit_slots_kernel) and lane-per-row
# halo clear (sx_zero_rows_kernel): partition tests + C4 at P = 1/2/4/8 (scripts/gpu_shard.sh),
# kernel stats at P = 8, then the frontier stall counters at the M = 20 distinct-batch launch
# with the locality layout (r04_pmc_frontier_layout_m20.txt; before: r04_pmc_frontier_distinct20.txt).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s7
mkdir -p $OUT
TAG=r04s7/shard bash scripts/gpu_shard.sh
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/shard_p8 -o run -- python3 bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/shard_p8.json 2> $OUT/shard_p8.err
echo "shard P=8 prof ok"
TAG=r04s7/pmc BENCH_ARGS="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2" bash scripts/pmc_frontier.sh
python scripts/pmc_summary.py gpurun_out/r04s7/pmc > $OUT/pmc_summary.txt 2>&1 || true
head -30 $OUT/pmc_summary.txt
