# Re-measure the secondary frontier workloads at the current defaults: C4, member-pool mode on
# C3, and the alert storm (C5).  TAG names the output directory.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-variants}
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config C4 --no-cpu-baseline --no-dropin --dense-steps 0 --steps 100 > $OUT/c4.json 2> $OUT/c4.err
echo "c4 ok"
timeout -k 10 200 python -u bench.py --pool --no-cpu-baseline --no-dropin --dense-steps 0 --steps 100 > $OUT/pool.json 2> $OUT/pool.err
echo "pool ok"
timeout -k 10 300 python -u bench.py --workload storm --no-cpu-baseline > $OUT/storm.json 2> $OUT/storm.err
echo "storm ok"
