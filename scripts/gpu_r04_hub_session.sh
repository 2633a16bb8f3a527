#!/bin/bash
# hub-order experiment + the RCCL world-size-1 test (one call)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04hub
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/r04hub/pytest_rccl.log 2>&1 && echo "rccl test ok" || { echo "rccl test FAILED"; tail -30 gpurun_out/r04hub/pytest_rccl.log; }
bash scripts/gpu_r04_hub.sh
