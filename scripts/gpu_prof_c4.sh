#!/bin/bash
# rocprofv3 kernel traces of the C4 and C3 frontier benches (round 2).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-profc4}
mkdir -p $OUT
B="--no-cpu-baseline --no-dropin --dense-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4 -o run -- python3 bench.py --config C4 --steps 10 --roofline-reps 5 $B > $OUT/c4.log 2>&1
echo "c4 prof ok"
find $OUT/c4 -name '*kernel_stats.csv' -exec head -12 {} \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o run -- python3 bench.py --no-cpu-baseline --no-dropin > $OUT/c3.log 2>&1
echo "c3 prof ok"
find $OUT/c3 -name '*kernel_stats.csv' -exec head -14 {} \;
