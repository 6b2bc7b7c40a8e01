# fp64 wave flush: its parity tests, then the fp64 bench line (T = 4) and its kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02_f64}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k "f64 or fp64 or deferred or per_scan or trajectory" > gpurun_out/$TAG/pytest.log 2>&1 && \
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --precision f64 --flush-interval 4 --no-cpu > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$TAG/kt -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --precision f64 --flush-interval 4 --no-cpu > gpurun_out/$TAG/kt.log 2>&1
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
