# Batches in flight (bench.py --pipeline P): ms per step at each P, two alternating passes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2; do
  for P in ${PIPES:-2 3 4 6}; do
    timeout -k 10 200 python -u bench.py --pipeline $P --no-cpu-baseline --no-dropin --dense-steps 0 --steps 200 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('P=$P', round(d['value']), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  done
done
