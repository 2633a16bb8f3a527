set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/alerts
timeout -k 10 300 python -u -m pytest tests/test_alerts_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/alerts/pytest.log 2>&1 || { tail -60 gpurun_out/alerts/pytest.log; exit 1; }
tail -15 gpurun_out/alerts/pytest.log
