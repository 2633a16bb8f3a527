#!/bin/bash
# PMC passes for the bench's kernels, one counter group per rocprofv3 run (gfx950 slot limits:
# FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2, so they get separate passes).  Run on the GPU box
# from the repo root.  Output: gpurun_out/pmc/<pass>/..._counter_collection.csv
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --no-cpu-baseline"}
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run l2 TCC_HIT_sum TCC_MISS_sum
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
