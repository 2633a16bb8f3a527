#!/bin/bash
# Round-2 measurements for DESIGN.md §10: C2 and C4 (9.9M-entry) frontier benches, the C4
# edge-cut path with the sparse and dense halo, the alert storm on one GPU and its
# fingerprint-sharded 2-rank path rehearsed on the one GPU (gloo).  Stops at the first failure.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r02m}
mkdir -p $OUT
B="--no-cpu-baseline --no-dropin --dense-steps 0"
timeout -k 10 300 python -u bench.py --config C2 $B > $OUT/c2.json 2> $OUT/c2.err
echo "C2"; cat $OUT/c2.json | head -c 600; echo
timeout -k 10 300 python -u bench.py --config C4 $B > $OUT/c4_frontier.json 2> $OUT/c4_frontier.err
echo "C4 frontier"; cat $OUT/c4_frontier.json | head -c 900; echo
for P in 1 2 4; do
  timeout -k 10 300 python -u bench.py --shard graph --config C4 --partitions $P --steps 5 --warmup 2 --no-cpu-baseline > $OUT/c4_shard_p$P.json 2> $OUT/c4_shard_p$P.err
  echo "C4 shard P=$P"; python3 -c "import json;d=json.load(open('$OUT/c4_shard_p$P.json'));c=d['config'];print(d['ms_per_step'], c['csr_entries'], c.get('halo_bytes_per_hop_max_rank'), c.get('halo_bytes_sent_per_hop_max_rank'), c.get('halo_reduction_vs_dense'))"
done
timeout -k 10 300 python -u bench.py --shard graph --config C4 --partitions 2 --steps 5 --warmup 2 --no-cpu-baseline --dense-halo > $OUT/c4_shard_p2_dense.json 2> $OUT/c4_shard_p2_dense.err
echo "C4 shard P=2 dense"; python3 -c "import json;d=json.load(open('$OUT/c4_shard_p2_dense.json'));print(d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --workload storm --steps 20 --warmup 3 > $OUT/storm_n1.json 2> $OUT/storm_n1.err
echo "storm N=1"; cat $OUT/storm_n1.json | head -c 1200; echo
EGRAPH_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --workload storm --gpus 2 --steps 20 --warmup 3 > $OUT/storm_n2_gloo1gpu.json 2> $OUT/storm_n2_gloo1gpu.err
echo "storm N=2 (gloo, one GPU)"; cat $OUT/storm_n2_gloo1gpu.json | head -c 1200; echo
