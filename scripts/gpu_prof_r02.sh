#!/bin/bash
# Frontier evidence at the current defaults: per-phase column profile and the counter passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-profr02}
mkdir -p $OUT
timeout -k 10 200 python -u scripts/frontier_profile.py > $OUT/phases.txt 2>&1
echo "phases ok"; tail -n 25 $OUT/phases.txt
TAG=${TAG:-profr02}/pmc bash scripts/pmc_frontier_r02.sh
