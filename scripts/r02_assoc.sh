# association iteration: the full GPU parity suite, then the phase probe and the driver bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r02_assoc}
mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 240 python scripts/assoc_probe.py 4096:8 4096:1 1024:8 > gpurun_out/$TAG/probe.txt 2>&1 && \
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
