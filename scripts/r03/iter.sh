# one iteration: GPU tests (optionally filtered), association phase stamps, driver-command bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_iter}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 240 python scripts/assoc_probe.py ${PROBE_CFGS:-4096:12 1024:8} > gpurun_out/$TAG/probe.txt 2>&1 || { echo "probe failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 200 --no-cpu > gpurun_out/$TAG/bench200.json 2>> gpurun_out/$TAG/bench.err
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
