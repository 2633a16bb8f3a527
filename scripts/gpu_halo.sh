#!/bin/bash
# Sparse vs dense halo exchange on the edge-cut C4 path (one GPU, P in-process partitions),
# plus the drop-in batcher tests (egr_rules_eval_staged).  Stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-halo}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_batcher_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
echo "tests ok"; tail -2 $OUT/pytest.log
for P in 2 4; do
  for mode in sparse dense; do
    timeout -k 10 300 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline $([ $mode = dense ] && echo --dense-halo) > $OUT/c4_p${P}_$mode.json 2> $OUT/c4_p${P}_$mode.err
    echo "P=$P $mode"; python3 -c "import json,sys; d=json.load(open('$OUT/c4_p${P}_$mode.json')); c=d['config']; print(d['ms_per_step'], c.get('halo_bytes_per_hop_max_rank'), c.get('halo_bytes_sent_per_hop_max_rank'), c.get('halo_reduction_vs_dense'))"
  done
done
