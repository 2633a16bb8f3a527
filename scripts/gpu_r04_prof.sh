#!/bin/bash
# Round 4: per-phase profile of the frontier kernel on the headline launch (20 different incident
# sets, layout on), rocprof kernel stats at the driver's settings (the device launch-order
# kernels included) and two bench runs.  Produces profiles/r04_frontier_phases_distinct20.txt,
# r04_kernel_stats_layout_s20.csv.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r04prof}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py tests/test_layout_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/bench$i.json 2> $OUT/bench$i.err
  python -c "import json;d=json.load(open('$OUT/bench$i.json'));r=d['roofline'];print('bench $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), round(r['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s20 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/prof_s20.log 2>&1
echo "prof ok"
find $OUT/prof_s20 -name '*kernel_stats.csv' | xargs -I{} sh -c 'head -12 {} | cut -c1-150'
timeout -k 10 300 python -u scripts/frontier_profile.py --merge 20 > $OUT/phases.txt 2> $OUT/phases.err
cat $OUT/phases.txt
