#!/bin/bash
# Round 4 session 12: the narrow table with interleaved buckets (keys + both score buffers per
# 48-B bucket: a probe returns the neighbour's score in the same LDS round trip) -- frontier
# parity tests on the default build (ILV on, 5 waves/SIMD, 27 VGPRs spilled), then an
# interleaved A/B: default vs exp_noilv (the round's layout) vs exp_ilv4 (ILV at 4 waves/SIMD).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s12
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_layout_gpu.py tests/test_frontier_scale_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
BA="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
L=kubernetes-aiops-evidence-graph_amd/lib
for i in 1 2; do
  for v in ilv noilv ilv4; do
    if [ $v = ilv ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 200 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
