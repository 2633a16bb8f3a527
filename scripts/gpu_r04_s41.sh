#!/bin/bash
# Round 4 session 41: check of the final tree (narrow table at seven workgroups per CU): the gpu
# suite, smoke, and the bench at its defaults and at --steps 20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04final6
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo "smoke ok"
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('bench', round(d['value']), round(d['ms_per_step'],5), round(r['frac'],4), round(r['avg_launch_ms'],4))"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin > $OUT/bench_s20.json 2> $OUT/bench_s20.err
python -c "import json;d=json.load(open('$OUT/bench_s20.json'));r=d['roofline'];print('s20', round(d['value']), round(d['ms_per_step'],5), round(r['frac'],4))"
