# one GPU iteration: parity tests, phase stamps, sequential + pipelined bench (no CPU baseline)
set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
echo "pytest exit $?" >> gpurun_out/gpu_tests.log
timeout -k 10 200 python scripts/scan_stamps.py > gpurun_out/stamps.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_seq.json 2> gpurun_out/bench_seq.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --pipeline 1 > gpurun_out/bench_pipe.json 2> gpurun_out/bench_pipe.err || exit 1
