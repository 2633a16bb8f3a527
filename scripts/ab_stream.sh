set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 100 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('side', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  EGRAPH_BENCH_ONE_STREAM=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 100 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('one ', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
mkdir -p gpurun_out/tl2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl2/prof -o run -- python3 bench.py --no-cpu-baseline --dense-steps 0 --steps 20 > /dev/null 2>&1
python scripts/timeline.py $(find gpurun_out/tl2/prof -name "*kernel_trace.csv") -3
