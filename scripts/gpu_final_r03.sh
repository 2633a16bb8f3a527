#!/bin/bash
# Round-3 final check of the committed tree: every GPU test, smoke, the bench at its defaults
# (400 steps: 50 batches per launch) and at the driver's --steps 20 --warmup 5 (20 per launch),
# rocprof stats of both (scripts/gpu_check_r03.sh), then the L2 request counters of the
# frontier at 50 batches per launch.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-final}
mkdir -p $OUT
TAG=${TAG:-final} bash scripts/gpu_check_r03.sh
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/rdreq -o rdreq -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 4 > $OUT/rdreq.log 2>&1
echo "rdreq pass ok"
