#!/bin/bash
# Quick GPU iteration on the frontier engine: its parity tests, the phase profile, one bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-fr}
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_frontier_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python -u scripts/frontier_profile.py --out $OUT/phases.json > $OUT/phases.log 2>&1
grep -v "^\[rank" $OUT/phases.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'frontier_ms',d['roofline']['avg_launch_ms'],'dense_ms',d.get('dense_engine',{}).get('ms_per_step'))"
