#!/bin/bash
# PMC HBM traffic passes (they refresh profiles/pmc_*.json, which the bench reads), then the
# GPU suite, smoke, the default bench and its rocprofv3 kernel-trace stats.  TAG names the run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-full}/pmc bash scripts/pmc_traffic.sh
TAG=${TAG:-full} bash scripts/gpu_check.sh
