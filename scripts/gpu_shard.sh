#!/bin/bash
# The edge-cut path (C4): the partition tests, then C4 at P = 1, 2, 4, 8 partitions in one
# process (per-partition compute times + the projected per-GPU step), fixed-capacity halo slots;
# P = 8 again with the host-read peer counts (A/B).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-shard}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_shard_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "shard or C4 or partition or fixed" > $OUT/pytest.log 2>&1
echo "tests ok"; tail -1 $OUT/pytest.log
show() {
  python -c "import json;d=json.load(open('$1'));c=d['config'];print('$2', round(d['ms_per_step'],2), 'ms in-process; partitions', [round(x,2) for x in c['partition_compute_ms']], 'critical', [round(x,2) for x in c.get('partition_critical_ms', [])], 'projected per GPU', round(c['projected_ms_per_gpu'],2), 'collectives', c.get('collectives_per_step'), 'at latency us', {k: round(v,2) for k,v in c.get('projected_ms_per_gpu_at_latency_us', {}).items()}, 'link B/step', c.get('link_bytes_per_step_max_rank'), 'slots', c.get('halo_slot_entries'), 'reruns', c.get('halo_overflow_reruns'))"
}
for P in 1 2 4 8; do
  timeout -k 10 200 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline > $OUT/c4_p$P.json 2> $OUT/c4_p$P.err
  show $OUT/c4_p$P.json "P=$P"
done
timeout -k 10 200 python -u bench.py --shard graph --config C4 --partitions 8 --steps 5 --warmup 2 --no-cpu-baseline --halo-host-counts > $OUT/c4_p8_hostcounts.json 2> $OUT/c4_p8_hostcounts.err
show $OUT/c4_p8_hostcounts.json "P=8 host-counts"
