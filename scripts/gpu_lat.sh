set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lat2
timeout -k 10 300 python -u -m pytest tests/test_batcher_gpu.py tests/test_rules_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lat2/pytest.log 2>&1
tail -1 gpurun_out/lat2/pytest.log
timeout -k 10 300 python -u scripts/latency_probe.py > gpurun_out/lat2/probe.txt 2>&1
cat gpurun_out/lat2/probe.txt
timeout -k 10 300 python -u scripts/frontier_profile.py > gpurun_out/lat2/phases.txt 2>&1
cat gpurun_out/lat2/phases.txt
