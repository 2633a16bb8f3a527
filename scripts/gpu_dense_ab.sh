#!/bin/bash
# Dense-engine A/B: the bench's dense step and hop launch (dense_engine) for the default build
# and each variant in $ALTS (scripts/build_variant.sh FILE=propagate.hip ...), interleaved, plus
# the C4 edge-cut at P = $SHARD_P (projected per-GPU step) when SHARD_P is set.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-dense_ab}
mkdir -p $OUT
for r in $(seq 1 ${REPS:-3}); do
  for a in base $ALTS; do
    if [ $a = base ]; then unset EGRAPH_LIB; n=base; else export EGRAPH_LIB=$PWD/$a; n=$(basename $(dirname $a)); fi
    timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-dropin --dense-steps 5 --roofline-reps 2 > $OUT/${n}_$r.json 2> $OUT/${n}_$r.err
    python -c "import json;d=json.load(open('$OUT/${n}_$r.json'))['dense_engine'];print('$n dense', round(d['ms_per_step'],4), 'hop', round(d['roofline']['avg_launch_ms'],4))"
    if [ -n "$SHARD_P" ]; then
      timeout -k 10 200 python bench.py --shard graph --config C4 --partitions $SHARD_P --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${n}_c4p${SHARD_P}_$r.json 2> $OUT/${n}_c4p${SHARD_P}_$r.err
      python -c "import json;c=json.load(open('$OUT/${n}_c4p${SHARD_P}_$r.json'))['config'];print('$n C4 P=$SHARD_P projected', round(c['projected_ms_per_gpu'],3), 'critical max', round(max(c['partition_critical_ms']),3))"
    fi
  done
done
