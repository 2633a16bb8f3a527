#!/bin/bash
# Round 4 session 36: rocprofv3 kernel stats of C4 through the replicated frontier on the closing
# tree (mid-first: fr_mid kernel + the wide retry of its overflows), --steps 20 --warmup 5.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s36
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4.json 2> $OUT/c4.err
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_c4.csv \;
rm -rf $OUT/prof
head -6 $OUT/kernel_stats_c4.csv | cut -c1-200
