#!/bin/bash
# Rehearse bench.py's multi-rank path on ONE GPU: N ranks share the device over gloo.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-ranks}
mkdir -p $OUT
for N in ${RANKS:-2 4}; do
  EGRAPH_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) \
    bench.py --gpus $N --steps 20 --warmup 3 --no-cpu-baseline --no-dropin \
    > $OUT/bench_n$N.json 2> $OUT/bench_n$N.err
  echo "N=$N ok"; cat $OUT/bench_n$N.json
done
