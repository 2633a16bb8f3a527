#!/bin/bash
# Round 4 session 21: tree with sparse hub chains + mid-first adapt(): the gpu suite, then the
# C3 headline at --steps 20 and C4 (adapt -> mid-first) at --steps 20.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s21
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
echo "gpu tests ok"; tail -1 $OUT/pytest_gpu.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$i.json 2> $OUT/c3_$i.err
python -c "import json;d=json.load(open('$OUT/c3_$i.json'));r=d['roofline'];print('C3', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])"
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_$i.json 2> $OUT/c4_$i.err
python -c "import json;d=json.load(open('$OUT/c4_$i.json'));r=d['roofline'];w=d['frontier_work'];print('C4', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'], w['overflowed'], w['global_columns'])"
done
