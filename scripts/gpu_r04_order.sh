#!/bin/bash
# Round 4: the many-block device launch order (grouped_cost_kernel + cost_order_kernel): the
# grouped-order tests, the headline bench, its kernel stats.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04order
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_layout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', int(d['value']), round(d['ms_per_step'],4))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/prof.log 2>&1
echo "prof ok"
head -8 $(find $OUT/prof -name "run_kernel_stats.csv" | head -1)
