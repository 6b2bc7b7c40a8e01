# the row-shard GPU tests, then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_shard}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_rowshard_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/$TAG/shard.log 2>&1 || { echo "shard failed" > gpurun_out/$TAG/status; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
