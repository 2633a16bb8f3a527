#!/bin/bash
# Round 3 session 3: storm + drop-in after the native keyed batch and entity assembly.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-s3e}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_storm_gpu.py tests/test_frontier_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
echo "storm ok"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 > $OUT/bench.json 2> $OUT/bench.err
echo "bench ok"
for K in 1 2 5 20; do
  timeout -k 10 120 python -u bench.py --steps $K --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench_k$K.json 2> $OUT/bench_k$K.err
  python -c "import json;d=json.load(open('$OUT/bench_k$K.json'));print('K=$K', round(d['ms_per_step']*$K,4), 'ms region')"
done
