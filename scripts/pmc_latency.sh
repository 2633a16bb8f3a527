#!/bin/bash
# Average in-flight latency of LDS and vector-memory instructions of the frontier kernel
# (Little's law: SQ_INST_LEVEL_x / SQ_INSTS_x), plus LDS conflict and wait counters.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-lat}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --dense-steps 0"}
run() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
run l1 SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
run l2 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
python3 scripts/pmc_summary.py $OUT frontier_lds_kernel
