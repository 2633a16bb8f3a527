# A/B a frontier environment switch: ENVVAR=1 vs unset, 3 alternating runs each
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('base', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
  env $ENVVAR=1 timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('$ENVVAR', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4))"
done
