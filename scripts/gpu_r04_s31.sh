#!/bin/bash
# Round 4 session 31: counters of the closing tree's frontier kernel at the M = 20 distinct-batch
# launch -- the stall / instruction / cache passes (scripts/pmc_frontier.sh; before:
# r04_pmc_frontier_distinct20.txt, r04_pmc_frontier_layout_m20.txt) and the bytes past L2
# (TCC_EA0_RDREQ, calibrated: pmc_frontier_calibrated_r04_distinct20_final2.json, which bench.py
# reads for roofline.traffic).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s31
mkdir -p $OUT
P="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
TAG=r04s31/pmc BENCH_ARGS="$P" bash scripts/pmc_frontier.sh
python scripts/pmc_summary.py gpurun_out/r04s31/pmc frontier_lds_kernel > $OUT/pmc_summary.txt 2>&1 || true
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/rdreq -o rdreq -- python3 bench.py $P > $OUT/rdreq.log 2>&1
echo "rdreq ok"
python scripts/pmc_rdreq.py $OUT/rdreq r04_distinct20_final2 C3 1024 20 20
cp profiles/pmc_frontier_calibrated_r04_distinct20_final2.json $OUT/
