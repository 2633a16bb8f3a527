#!/bin/bash
# Round 4 session 13: code size of the narrow frontier kernel (23.2k -> 7.4k instructions: one
# CAS site per insert, the probe batches as a rolled loop): frontier parity tests on the default
# build, an interleaved A/B of default vs exp_cas1 (the single CAS site only) vs exp_base (the
# round's kernel), and instruction-cache counters on base and default (if gfx950 exposes them).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s13
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_frontier_gpu.py tests/test_configs_gpu.py tests/test_layout_gpu.py tests/test_frontier_scale_gpu.py tests/test_storm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
BA="--steps 20 --warmup 5 --no-cpu-baseline --no-dropin --dense-steps 0"
L=kubernetes-aiops-evidence-graph_amd/lib
for i in 1 2; do
  for v in small cas1 base; do
    if [ $v = small ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
    timeout -k 10 200 python bench.py $BA > $OUT/$v$i.json 2> $OUT/$v$i.err
    python -c "import json;d=json.load(open('$OUT/$v$i.json'));r=d['roofline'];print('$v $i', round(d['value']), round(d['ms_per_step'],4), round(r['avg_launch_ms'],4))" | tee -a $OUT/ab.txt
  done
done
unset EGRAPH_LIB
PA="--steps 2 --warmup 1 --merge 20 --no-cpu-baseline --no-dropin --dense-steps 0 --roofline-reps 2"
for v in small base; do
  if [ $v = small ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/pmc_$v -o sq -- python3 bench.py $PA > $OUT/pmc_$v.log 2>&1 && echo "pmc $v ok" || echo "pmc $v failed"
  python scripts/pmc_summary.py $OUT/pmc_$v frontier_lds_kernel | tee -a $OUT/pmc.txt
done
unset EGRAPH_LIB
for v in small base; do
  if [ $v = small ]; then unset EGRAPH_LIB; else export EGRAPH_LIB=$PWD/$L/exp_$v/libegraph.so; fi
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS --output-format csv -d $OUT/ic_$v -o ic -- python3 bench.py $PA > $OUT/ic_$v.log 2>&1 && python scripts/pmc_summary.py $OUT/ic_$v frontier_lds_kernel | tee -a $OUT/pmc.txt || echo "icache counters unavailable ($v)"
done
unset EGRAPH_LIB
