#!/bin/bash
# Round 4 session 38: the closing check of the tree with the one-buffer mid table (gpu tests,
# smoke, bench at its defaults and at --steps 20, rocprof of both; C4; the storm), then the
# narrow table with one score buffer at six workgroups per CU (exp_n6) against it on C3.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=r04final4 bash scripts/gpu_check.sh
OUT=gpurun_out/r04final4
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4_prof.json 2> $OUT/c4_prof.err
find $OUT/prof_c4 -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats_c4.csv \;
rm -rf $OUT/prof_c4
timeout -k 10 300 python bench.py --config C4 --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c4.json 2> $OUT/c4.err
python -c "import json;d=json.load(open('$OUT/c4.json'));r=d['roofline'];print('C4', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4), d['config']['first_table'])"
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));print('storm', round(d['value']), d['unit'], round(d['ms_per_step'],3))"
L=$PWD/kubernetes-aiops-evidence-graph_amd/lib
EGRAPH_LIB=$L/exp_n6/libegraph.so timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_n6.log 2>&1
echo "n6 parity: $(tail -1 $OUT/pytest_n6.log)" | tee -a $OUT/ab.txt
for i in 1 2; do
  for v in base n6; do
    if [ $v = base ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$L/exp_$v/libegraph.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0 > $OUT/c3_$v$i.json 2> $OUT/c3_$v$i.err
    python -c "import json;d=json.load(open('$OUT/c3_$v$i.json'));r=d['roofline'];print('C3 $v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
