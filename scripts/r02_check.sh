# GPU tests (incl. the bench-configuration parity), the driver's bench command, and its
# kernel-trace summary; each GPU step under its own limit, chained so a failure stops the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02b}
mkdir -p gpurun_out/$TAG
rm -f gpurun_out/bench_config_parity.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/$TAG/kt.log 2>&1
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
