#!/bin/bash
# Round 3: batches per launch (--merge M, one stream per lane) against lanes (--pipeline P) and
# HIP's hardware queues per process, ms/step at the bench defaults, one box.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-merge_r03}
mkdir -p $OUT
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 150 python -u bench.py --steps ${STEPS:-240} --no-cpu-baseline --no-dropin --dense-steps 0 $ARGS > $OUT/$name.json 2> $OUT/$name.err
  python -c "import json;d=json.load(open('$OUT/$name.json'));r=d['roofline'];print('$name', round(d['ms_per_step'],4), round(d['value']/1e6,2), 'launch_ms', round(r['avg_launch_ms'],4))"
}
if [ -z "$SWEEP2" ]; then
for M in 1 2 3 4 6; do ARGS="--pipeline 1 --merge $M" run p1_m$M; done
for M in 2 4; do ARGS="--pipeline 2 --merge $M" run p2_m$M; done
ARGS="--pipeline 3 --merge 1" run p3_m1
for Q in 1 2; do ARGS="--pipeline 1 --merge 4" run p1_m4_q$Q GPU_MAX_HW_QUEUES=$Q; done
else
# larger groups on one stream, and their hardware-queue sensitivity
for M in 8 12 16 24; do ARGS="--pipeline 1 --merge $M" run p1_m$M; done
for Q in 1 2; do ARGS="--pipeline 1 --merge 16" run p1_m16_q$Q GPU_MAX_HW_QUEUES=$Q; done
ARGS="--pipeline 2 --merge 8" run p2_m8
ARGS="--pipeline 2 --merge 8" run p2_m8_q1 GPU_MAX_HW_QUEUES=1
fi
