#!/bin/bash
# Round 4 session 42: C4 through the replicated frontier and the storm bench on the final tree.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04final6
mkdir -p $OUT
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4.json 2> $OUT/c4.err
python -c "import json;d=json.load(open('$OUT/c4.json'));r=d['roofline'];print('C4', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])"
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));print('storm', round(d['value']), d['unit'], round(d['ms_per_step'],3))"
