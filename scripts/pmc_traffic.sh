#!/bin/bash
# HBM traffic of the bench kernels (MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE and
# WRITE_SIZE in separate passes; gfx950 FETCH_SIZE counts half the bytes of 16-B/lane reads).
# Runs the default frontier bench plus a few dense steps, so both engines' kernels appear.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-traffic}
mkdir -p $OUT
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --dense-steps 3 --no-cpu-baseline"}
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 bench.py $ARGS > $OUT/$name.log 2>&1
  echo "pass $name ok"
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run rdreq TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
python3 scripts/pmc_summary.py $OUT frontier_lds_kernel "hop_kernel<32, false>" reach_kernel
python3 scripts/pmc_traffic.py $OUT
cp profiles/pmc_frontier.json profiles/pmc_hop.json $OUT/
