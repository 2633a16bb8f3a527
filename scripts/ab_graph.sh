set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('graph  ', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['frontier_work']['members'])"
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --dense-steps 0 --steps 200 --no-graph 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print('nograph', round(d['ms_per_step'],4), round(d['roofline']['avg_launch_ms'],4), d['frontier_work']['members'])"
done
