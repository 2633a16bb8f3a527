#!/bin/bash
# Round 3: storm + drop-in after the concatenating seed-key assembly: their GPU tests, the storm
# bench twice, the drop-in numbers.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-storm3}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_storm_gpu.py tests/test_configs_gpu.py tests/test_graph_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm$rep.json 2> $OUT/storm$rep.err
  python -c "import json;d=json.load(open('$OUT/storm$rep.json'));c=d['config'];print('storm', round(d['value']), round(d['ms_per_step'],2), c['stage_ms_mean'], c['reseed_per_tick'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));g=d['dropin_graph'];r=d['dropin_rules'];print('bench', round(d['value']/1e6,2), 'graph', round(g['value']), round(g['ms_per_batch'],2), g['matches_engine_topk'], 'rules', round(r['value']), 'conc', round(r['concurrent']['value']))"
