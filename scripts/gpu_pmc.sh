#!/bin/bash
# Counter passes over the bench's kernels at the driver's workload (--steps 20 --warmup 5), one
# counter group per rocprofv3 run (gfx950 slots: 8 SQ, 4 TCC, 4 TCP; FETCH_SIZE takes 3 TCC,
# WRITE_SIZE 2), each under its own KILL time limit.  Then:
#   scripts/pmc_summary.py   -> $OUT/summary.txt (per-dispatch sums per kernel)
#   scripts/pmc_rdreq.py     -> profiles/pmc_frontier_calibrated_$PMC_TAG.json (bytes past L2 per
#                               narrow frontier launch, stamped with the libegraph.so build hash)
#   scripts/pmc_traffic.py   -> profiles/pmc_hop.json (dense hop HBM bytes, stamped)
# bench.py reports either file's bytes as roofline.traffic only while it loads the same build.
# Env: TAG (output dir), PMC_TAG (profile name), PASSES (subset), BENCH_ARGS, EGRAPH_LIB (variant).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 3 --roofline-reps 2"}
PASSES=${PASSES:-"rdreq fetch write sq1 sq2 tcc tcp"}
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
for p in $PASSES; do
  case $p in
    rdreq) run rdreq TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum ;;
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    sq1) run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU ;;
    sq2) run sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_WR ;;
    sq3) run sq3 ${SQ3:-SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE} ;;
    # active lanes per VALU instruction: SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64)
    lanes) run lanes SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU ;;
    tcc) run tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum ;;
    tcp) run tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum ;;
  esac
done
python3 scripts/pmc_summary.py $OUT frontier_lds_kernel frontier_lds_retry_kernel "hop_kernel<32, false, " > $OUT/summary.txt
cat $OUT/summary.txt
if [ -n "$PMC_TAG" ] && [ -d $OUT/rdreq ]; then
  python3 scripts/pmc_rdreq.py $OUT/rdreq $PMC_TAG ${PMC_CONFIG:-C3} 1024 20 20 > /dev/null
  cp profiles/pmc_frontier_calibrated_$PMC_TAG.json $OUT/
fi
if [ -n "$PMC_TAG" ] && [ -d $OUT/fetch ] && [ -d $OUT/write ]; then
  python3 scripts/pmc_traffic.py $OUT > /dev/null
  cp profiles/pmc_hop.json $OUT/
fi
