#!/bin/bash
# A/B bench configurations in one GPU call: CFG holds one variant per line,
#   name|ENV=val ENV2=val|extra bench args
# run REPS times interleaved; each run under its own time limit.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-abc}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-2}); do
  while IFS='|' read -r name envs args; do
    [ -z "$name" ] && continue
    eval env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-dropin --dense-steps 0 ${BENCH_ARGS:-} $args > $OUT/$name.$r.json 2> $OUT/$name.$r.err
    python -c "import json;d=json.load(open('$OUT/$name.$r.json'));r=d['roofline'];print('$name rep $r', round(d['value']), round(d['ms_per_step'],4), 'launch', round(r['avg_launch_ms'],4))"
  done <<< "$CFG"
done
