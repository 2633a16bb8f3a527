#!/bin/bash
# One GPU call for the edge-cut partitioned path: its GPU tests, then the C4
# --shard graph bench with P in-process partitions on the one GPU, and the C4 replicated
# frontier bench for comparison.  Each GPU step has its own limit; the chain stops on failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-shard}
mkdir -p $OUT
timeout -k 10 240 python -u -m pytest tests/test_shard_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_shard.log 2>&1
echo "shard tests ok"; tail -2 $OUT/pytest_shard.log
for P in ${PARTS:-1 2 4}; do
  timeout -k 10 300 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 $([ $P = 1 ] || echo --no-cpu-baseline) ${XARGS:-} > $OUT/bench_c4_p$P.json 2> $OUT/bench_c4_p$P.err
  echo "P=$P"; cat $OUT/bench_c4_p$P.json
done
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --dense-steps 0 > $OUT/bench_c4_frontier.json 2> $OUT/bench_c4_frontier.err
echo "C4 frontier"; cat $OUT/bench_c4_frontier.json
