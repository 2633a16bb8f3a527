#!/bin/bash
# One GPU call: gpu tests + bench only (no profiler).  TAG names the output directory.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
