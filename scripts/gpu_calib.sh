#!/bin/bash
# TCC_EA0_RDREQ per 128-B line for the frontier's access widths (scripts/calib_gather.hip),
# then the frontier kernel's own requests and write requests in separate passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-calib}
mkdir -p $OUT
B=kubernetes-aiops-evidence-graph_amd/lib/calib_gather
timeout -k 10 60 $B > $OUT/calib.txt
cat $OUT/calib.txt
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/rd -o rd -- $B > $OUT/rd.log 2>&1
echo "pass rd ok"
python3 scripts/pmc_summary.py $OUT/rd stream16 stride_kernel random8 flush
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $OUT/frd -o frd -- python3 bench.py $ARGS > $OUT/frd.log 2>&1
echo "pass frd ok"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/fwr -o fwr -- python3 bench.py $ARGS > $OUT/fwr.log 2>&1
echo "pass fwr ok"
python3 scripts/pmc_summary.py $OUT frontier_lds_kernel
