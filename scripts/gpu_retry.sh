#!/bin/bash
# The wide-table retry grid and the native sparse halo: parity tests, then C4 / C3 benches and
# the C4 edge-cut benches (sparse and dense halo).  Stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-retry}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_frontier_gpu.py tests/test_frontier_scale_gpu.py tests/test_configs_gpu.py tests/test_shard_gpu.py -x -v --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
B="--no-cpu-baseline --no-dropin --dense-steps 0"
timeout -k 10 300 python -u bench.py --config C4 $B > $OUT/c4.json 2> $OUT/c4.err
python3 -c "import json;d=json.load(open('$OUT/c4.json'));print('C4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['frontier_work'])"
timeout -k 10 300 python -u bench.py $B > $OUT/c3.json 2> $OUT/c3.err
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('C3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['rules_kernel']['isolated_us_median'])"
for P in 2 4; do
  for mode in sparse dense; do
    timeout -k 10 300 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline $([ $mode = dense ] && echo --dense-halo) > $OUT/c4_p${P}_$mode.json 2> $OUT/c4_p${P}_$mode.err
    python3 -c "import json; d=json.load(open('$OUT/c4_p${P}_$mode.json')); c=d['config']; print('P=$P $mode', d['ms_per_step'], c.get('halo_bytes_per_hop_max_rank'), c.get('halo_bytes_sent_per_hop_max_rank'), c.get('halo_reduction_vs_dense'))"
  done
done
