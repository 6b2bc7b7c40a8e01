# full GPU suite (product build), smoke, then the driver-command bench with its CPU legs
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_full}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
