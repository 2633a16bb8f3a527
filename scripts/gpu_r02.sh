#!/bin/bash
# Round-2 GPU call: gpu tests, smoke, bench (default + batch / pipeline variants), rocprofv3
# kernel-trace stats of the default bench.  Each GPU step under its own limit; stop at the first
# failure (set -e).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke ok"
fi
timeout -k 10 300 python -u bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"; cat $OUT/bench.json
for v in ${VARIANTS:-}; do
  a=${v//,/ }
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-dropin --dense-steps 0 $a > $OUT/bench_${v//[ ,-]/_}.json 2> $OUT/bench_${v//[ ,-]/_}.err
  echo "variant $a"; cat $OUT/bench_${v//[ ,-]/_}.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
if [ -z "$SKIP_PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-dropin ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
echo "prof ok"
find $OUT/prof -name '*kernel_stats.csv' -exec cat {} \;
fi
