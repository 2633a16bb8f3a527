#!/bin/bash
# Dense-path round: the dense / partitioned parity tests, the C3 bench's dense engine with and
# without the zero-tile skip, then the C4 edge-cut breakdown at P = 1 and 8.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-dense}; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_graph_gpu.py tests/test_shard_gpu.py tests/test_update_gpu.py tests/test_ops_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests: $(tail -1 $OUT/pytest.log)"
for alt in skip noskip; do
  if [ $alt = noskip ]; then export EGRAPH_HOP_NO_SKIP=1; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 5 > $OUT/bench_$alt.json 2> $OUT/bench_$alt.err
  python -c "import json;d=json.load(open('$OUT/bench_$alt.json'))['dense_engine'];print('$alt dense', round(d['ms_per_step'],3), 'ms/step hop', round(d['roofline']['avg_launch_ms'],4), 'ms frac', round(d['roofline']['frac'],3))"
  unset EGRAPH_HOP_NO_SKIP
done
TAG=${TAG:-dense}/shard bash scripts/gpu_shard_breakdown.sh
