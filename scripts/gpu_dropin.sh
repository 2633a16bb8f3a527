#!/bin/bash
# Drop-in rules path: the single-call latency breakdown and the bench's drop-in figures.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-dropin}
mkdir -p $OUT
timeout -k 10 300 python -u scripts/latency_probe.py > $OUT/latency.txt 2>&1
echo "probe ok"; cat $OUT/latency.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --steps 50 > $OUT/bench.json 2> $OUT/bench.err
python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step']);print(json.dumps(d['dropin_rules']))"
