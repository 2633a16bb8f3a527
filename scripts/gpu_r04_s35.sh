#!/bin/bash
# Round 4 session 35: the closing check of the tree with the wide table's light-row treatment
# (scripts/gpu_check.sh: gpu tests, smoke, bench at its defaults and at --steps 20, rocprof of
# both), then C4 through the replicated frontier and the storm bench.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r04final3 bash scripts/gpu_check.sh
OUT=gpurun_out/r04final3
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4.json 2> $OUT/c4.err
python -c "import json;d=json.load(open('$OUT/c4.json'));r=d['roofline'];print('C4', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])"
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));print('storm', round(d['value']), d['unit'], round(d['ms_per_step'],3))"
