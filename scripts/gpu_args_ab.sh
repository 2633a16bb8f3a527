#!/bin/bash
# A/B of bench.py command-line settings on one box, interleaved: ARGS_ALTS="name:--flag value,..."
# (commas separate the flags of one alternative), each against the driver's --steps 20
# --warmup 5 line, REPS rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-argsab}; mkdir -p $OUT
BASE="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 5"
for r in $(seq 1 ${REPS:-3}); do
  for a in "base:" $ARGS_ALTS; do
    n=${a%%:*}; extra=$(echo "${a#*:}" | tr ',' ' ')
    timeout -k 10 200 python bench.py $BASE $extra > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err
    python -c "import json;d=json.load(open('$OUT/${n}_$r.json'));c=d['config'];print('$n', round(d['value']), round(d['ms_per_step'],5), 'lanes', c['lanes'], 'M', c['batches_per_launch'])"
  done
done
