#!/bin/bash
# Round 4 session 29: per-column phase times with light-row tails + retry queue (closing tree) -- mid
# C4 (mid-first) and the C3 headline launch (narrow), 20 distinct batches each.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r04s29
mkdir -p $OUT
timeout -k 10 300 python scripts/frontier_profile.py --config C4 --merge 20 --out $OUT/c4.json > $OUT/c4.txt 2>&1
timeout -k 10 300 python scripts/frontier_profile.py --config C3 --merge 20 --out $OUT/c3.json > $OUT/c3.txt 2>&1
