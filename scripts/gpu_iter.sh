# one GPU iteration: all parity tests, scan phase stamps, then benches (stops at the first failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for t in 1 4; do T=$t timeout -k 10 120 python scripts/scan_stamps.py || exit 1; done
for cfg in ${BENCH_CFGS:-"0 1" "0 4" "1 4"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-cpu --pipeline $1 --flush-interval $2 > gpurun_out/bench_p$1_t$2.json 2> gpurun_out/bench_p$1_t$2.err || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_p$1_t$2.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_p$1_t$2.json')); print('$cfg', round(d['value']), round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, round(d['roofline']['hbm_frac'],3), round(d['roofline']['mfma_frac'],3), d['all_lines_matched'])"
done
