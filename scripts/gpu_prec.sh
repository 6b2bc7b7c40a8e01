set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for pr in f32 f16 f64; do for t in 1 4; do
  timeout -k 10 200 python bench.py --no-cpu --precision $pr --flush-interval $t > gpurun_out/b_$pr_$t.json 2> gpurun_out/b.err || { echo "bench failed"; tail -20 gpurun_out/b.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/b_$pr_$t.json')); print('$pr', $t, round(d['value']), round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, round(d['roofline']['hbm_frac'],3), round(d['roofline']['mfma_frac'],3), d['all_lines_matched'])"
done; done
