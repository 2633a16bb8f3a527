#!/bin/bash
# Round-2 counter passes over the bench's frontier kernel, one counter group per rocprofv3 run
# (kernel dispatches are serialised under --pmc, so these are per-launch figures of a launch
# that has the GPU to itself): L2 (TCC) hit rate, L1 (TCP) -> L2 request latency, wave
# wait/busy cycles, LDS and vector-memory instruction levels (Little's law latency).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmcf}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"}
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum
run l1 SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU
run l2 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU
python3 scripts/pmc_summary.py $OUT frontier_lds_kernel > $OUT/summary.txt
cat $OUT/summary.txt
