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
