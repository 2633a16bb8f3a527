#!/bin/bash
# One GPU call: gpu tests, smoke, bench, rocprofv3 kernel-trace stats of the bench.
# Every GPU step runs under its own time limit; the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
echo "prof ok"
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
