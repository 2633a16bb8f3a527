#!/bin/bash
# A/B of two _egr_pyhost builds on the encoder (scripts/encode_threads.py), interleaved.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do
  for v in default ${ALT:-exp_pyhost_old}; do
    if [ $v = default ]; then unset EGRAPH_PYHOST_DIR; else export EGRAPH_PYHOST_DIR=$PWD/kubernetes-aiops-evidence-graph_amd/lib/$v; fi
    echo "$v: $(timeout -k 10 120 python -u scripts/encode_threads.py 16 2>&1 | grep threads)"
  done
done
