#!/bin/bash
# Round-3 closing check after the concatenating seed-key assembly (pyhost.seed_keys): every GPU
# test, smoke, the bench at its defaults and at --steps 20 --warmup 5, rocprof stats of both
# (scripts/gpu_check_r03.sh), then the storm bench once.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-final2}
mkdir -p $OUT
TAG=${TAG:-final2} bash scripts/gpu_check_r03.sh
timeout -k 10 300 python -u bench.py --workload storm > $OUT/storm.json 2> $OUT/storm.err
python -c "import json;d=json.load(open('$OUT/storm.json'));c=d['config'];print('storm', round(d['value']), round(d['ms_per_step'],2), c['stage_ms_mean'], c['reseed_per_tick'])"
