# one GPU iteration: parity tests, then benches over (pipeline, flush interval); stops at the first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
for cfg in "0 1" "1 1" "0 4" "1 4" "0 8" "1 8" "0 16"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --pipeline $1 --flush-interval $2 > gpurun_out/bench_p$1_t$2.json 2> gpurun_out/bench_p$1_t$2.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_p$1_t$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_p$1_t$2.json')); print('$cfg', round(d['value']), d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['all_lines_matched'])"
done
