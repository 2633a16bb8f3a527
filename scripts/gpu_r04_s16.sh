#!/bin/bash
# Round 4 session 16: claimed member chunks in the frontier's row phases (a wave takes the next
# chunk from an LDS counter instead of a fixed stripe, so the phase barrier waits less for the
# wave that drew the hubs): parity tests on the default build (claimed), interleaved A/B against
# exp_static (the fixed stripes), and the per-phase profile of the default build.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s16
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_layout_gpu.py tests/test_frontier_scale_gpu.py tests/test_storm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
BA="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
L=kubernetes-aiops-evidence-graph_amd/lib
for i in 1 2 3; do
  for v in dyn static; do
    if [ $v = dyn ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 200 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
timeout -k 10 300 python -u scripts/frontier_profile.py --merge 20 > $OUT/phases.txt 2> $OUT/phases.err || echo "profile failed"
head -30 $OUT/phases.txt
