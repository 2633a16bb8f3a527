#!/bin/bash
# The closing check of a tree (one GPU call): gpu tests, smoke, the bench at its defaults and at the driver's short settings
# (--steps 20 --warmup 5), rocprofv3 kernel-trace stats of both.  Every GPU step runs under its
# own time limit; the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-check}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
  echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  echo "smoke ok"
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin ${BENCH_ARGS:-} > $OUT/bench_s20.json 2> $OUT/bench_s20.err
echo "bench s20 ok"; cat $OUT/bench_s20.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-dropin ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
echo "prof ok"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} > $OUT/prof_s20.log 2>&1
echo "prof s20 ok"
find $OUT/prof $OUT/prof_s20 -name '*kernel_stats.csv' | xargs -I{} sh -c 'echo {}; head -6 {} | cut -c1-160'
