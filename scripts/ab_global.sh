# A/B the overflow fallback launch: EGRAPH_FRONTIER_AB_GLOBAL unset (wide 512-thread grid),
# 1 (256-thread grid), 3 (64-thread grid, the default)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  for v in 0 1 3; do
    EGRAPH_FRONTIER_AB_GLOBAL=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('global=$v', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['frontier_work']['overflowed'])"
  done
done
for v in 1 3; do
  EGRAPH_FRONTIER_AB_GLOBAL=$v timeout -k 10 300 python -u -m pytest tests/test_frontier_scale_gpu.py tests/test_frontier_gpu.py -m gpu -x -q --durations=4 --timeout 120 --timeout-method thread > gpurun_out/ab_global_tests_$v.log 2>&1
  echo "tests global=$v ok"; tail -1 gpurun_out/ab_global_tests_$v.log
done
