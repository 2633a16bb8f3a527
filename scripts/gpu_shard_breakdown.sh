#!/bin/bash
# C4 edge-cut at P = 1 and 8 (one process): per-partition critical path with the slowest
# partition's calls broken down by chain and kind (bench.py config.slowest_partition_breakdown_ms)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-shardbd}
mkdir -p $OUT
for P in ${PS:-1 8}; do
  timeout -k 10 200 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/c4_p$P.json 2> $OUT/c4_p$P.err
  python -c "import json;c=json.load(open('$OUT/c4_p$P.json'))['config'];print('P=$P projected', round(c['projected_ms_per_gpu'],3), 'crit', [round(x,2) for x in c['partition_critical_ms']], 'halo/owned', c['halo_over_owned']);[print('   ',k,v) for k,v in c['slowest_partition_breakdown_ms'].items()]"
done
