#!/bin/bash
# Round 3: batches in flight (--pipeline P) and HIP's hardware queues per process
# (GPU_MAX_HW_QUEUES) against ms/step at the bench defaults, one box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pipe_r03}
mkdir -p $OUT
for P in 2 3 4 6; do
  timeout -k 10 120 python -u bench.py --pipeline $P --steps 200 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/p$P.json 2> $OUT/p$P.err
  python -c "import json;d=json.load(open('$OUT/p$P.json'));print('P=$P queues=default', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
done
for Q in 1 2 3; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python -u bench.py --steps 200 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/q$Q.json 2> $OUT/q$Q.err
  python -c "import json;d=json.load(open('$OUT/q$Q.json'));print('P=3 queues=$Q', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
done
# the seed input: resident grouped seeds + host launch order (default) against the device sort
for SI in sort grouped; do
  timeout -k 10 120 python -u bench.py --seed-input $SI --steps 200 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/si_$SI.json 2> $OUT/si_$SI.err
  python -c "import json;d=json.load(open('$OUT/si_$SI.json'));print('P=3 seed-input=$SI', round(d['ms_per_step'],4), round(d['value']/1e6,2))"
done
