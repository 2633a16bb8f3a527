#!/bin/bash
# A/B of the counter clearing at the driver's --steps 20: the default build (one clear kernel)
# against lib/exp_base (two fill nodes, HEAD's frontier.hip), interleaved; frontier GPU tests first.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abclear}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then export EGRAPH_LIB=$PWD/kubernetes-aiops-evidence-graph_amd/lib/exp_base/libegraph.so; else unset EGRAPH_LIB; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/$v$rep.json 2> $OUT/$v$rep.err
    python -c "import json;d=json.load(open('$OUT/$v$rep.json'));r=d['roofline'];print('$v', round(d['value']/1e6,3), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['in_region']['span_ms_mean'],4))"
  done
done
