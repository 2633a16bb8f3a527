#!/bin/bash
# The host-heavy workloads beside the headline: C4 through the replicated frontier (mid-first
# after adapt(), 20 distinct batches per launch) with its rocprof kernel stats, and the C5 alert
# storm on one GPU.  Every GPU step under its own time limit; the chain stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-storm}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4.json 2> $OUT/c4.err
python -c "import json;d=json.load(open('$OUT/c4.json'));r=d['roofline'];print('C4', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])"
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_prof.json 2> $OUT/c4_prof.err
  find $OUT/prof_c4 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_c4.csv \;
  rm -rf $OUT/prof_c4
fi
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));print('storm', round(d['value']), d['unit'], round(d['ms_per_step'],3))"
