#!/bin/bash
# Round 4 session 18: where the C4 replicated-frontier step goes with the mid-first geometry
# ($EGRAPH_FRONTIER_MID=1): rocprof kernel split (mid kernel vs the wide retry of its overflows)
# and per-column phase times / member counts of the mid kernel.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s18
mkdir -p $OUT
export EGRAPH_FRONTIER_MID=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench.json 2> $OUT/bench.err
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_mid.csv \;
timeout -k 10 300 python scripts/frontier_profile.py --config C4 --merge 20 --out $OUT/phases.json > $OUT/phases.txt 2>&1
unset EGRAPH_FRONTIER_MID
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof2 -o run -- python3 bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench_wide.json 2> $OUT/bench_wide.err
find $OUT/prof2 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_wide.csv \;
rm -rf $OUT/prof $OUT/prof2
