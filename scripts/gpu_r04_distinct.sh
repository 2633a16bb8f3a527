#!/bin/bash
# Round 4, verdict item 1: the headline with M DIFFERENT incident sets per launch against round
# 3's M copies of one set, at the driver's settings (--steps 20 --warmup 5): bench JSON of both,
# rocprofv3 kernel stats of the distinct run, TCC_EA0_RDREQ (bytes past L2) of both and the
# stall counters of the distinct run.  Produces profiles/r04_distinct_*.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r04d}
mkdir -p $OUT
S20="--steps 20 --warmup 5"
timeout -k 10 300 python -u bench.py $S20 > $OUT/bench_s20.json 2> $OUT/bench_s20.err
echo "bench distinct ok"; cat $OUT/bench_s20.json | cut -c1-600
timeout -k 10 200 python -u bench.py $S20 --replicate-batches --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench_s20_rep.json 2> $OUT/bench_s20_rep.err
echo "bench replicated ok"; cut -c1-300 $OUT/bench_s20_rep.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s20 -o run -- python3 bench.py $S20 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/prof_s20.log 2>&1
echo "prof ok"
P="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/rdreq -o rdreq -- python3 bench.py $P > $OUT/rdreq.log 2>&1
echo "rdreq distinct ok"
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/rdreq_rep -o rdreq -- python3 bench.py $P --replicate-batches > $OUT/rdreq_rep.log 2>&1
echo "rdreq replicated ok"
for pass in "sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
            "sq2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_WR" \
            "tcc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
            "tcp TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  set -- $pass; name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o $name -- python3 bench.py $P > $OUT/pmc_$name.log 2>&1
  echo "pmc $name ok"
done
python scripts/pmc_rdreq.py $OUT/rdreq r04_distinct20 C3 1024 20 20
python scripts/pmc_rdreq.py $OUT/rdreq_rep r04_replicated20 C3 1024 20 1
python scripts/pmc_summary.py $OUT/pmc_sq1 frontier_lds_kernel > $OUT/pmc_stalls.txt
for d in sq2 tcc tcp; do python scripts/pmc_summary.py $OUT/pmc_$d frontier_lds_kernel >> $OUT/pmc_stalls.txt; done
cat $OUT/pmc_stalls.txt
find $OUT/prof_s20 -name '*kernel_stats.csv' | xargs -I{} sh -c 'echo {}; head -6 {} | cut -c1-160'
