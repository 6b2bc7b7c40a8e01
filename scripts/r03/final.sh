# round-end check on the final tree: GPU suite, smoke, the driver's bench command, counter profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_final}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 || { echo "pytest failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$TAG/smoke.log 2>&1 || { echo "smoke failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "bench failed" > gpurun_out/$TAG/status; exit 1; }
PREFIX=${TAG} PROF_SET="${PROF_SET:-n4096 n1024}" bash scripts/r03/profiles.sh || { echo "profiles failed" > gpurun_out/$TAG/status; exit 1; }
echo ok > gpurun_out/$TAG/status
