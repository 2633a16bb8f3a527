#!/bin/bash
# The merged single-stream schedule: its parity tests, the frontier's read / write requests
# past L2 per launch at the bench default (M = 20 for --steps 20 and 400), then the bench and
# rocprof stats (scripts/gpu_check_r03.sh without the full test suite).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-mcheck}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py tests/test_bench_dist.py -m gpu -x -v --timeout 150 --timeout-method thread -k "bench_config" > $OUT/pytest_merge.log 2>&1
echo "merge tests ok"; tail -3 $OUT/pytest_merge.log
SKIP_TESTS=1 TAG=${TAG:-mcheck} bash scripts/gpu_check_r03.sh
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d $OUT/rdreq -o rdreq -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 4 > $OUT/rdreq.log 2>&1
echo "rdreq pass ok"
python3 scripts/pmc_rdreq.py $OUT/rdreq merge20 C3 1024 20
