#!/bin/bash
# Round 3 session 3: the region-length curve of the default bench (fixed overhead vs steady
# state), the drop-in numbers with the native seed attachment, and the storm at its defaults.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-s3a}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu-baseline --dense-steps 0 > $OUT/bench_dropin.json 2> $OUT/bench_dropin.err
echo "dropin ok"
for K in 20 50 100 200; do
  timeout -k 10 120 python -u bench.py --steps $K --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench_k$K.json 2> $OUT/bench_k$K.err
  echo "k$K ok"
done
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
echo "storm ok"
