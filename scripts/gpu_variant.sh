# flush-kernel variant A/B: parity with the default selection, then bench sweep (stops at first failure)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "deferred or per_scan or n4096 or trajectory or map or edge" > gpurun_out/var_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/var_tests.log; exit 1; }
tail -2 gpurun_out/var_tests.log
for v in ${VARIANTS:-0 3}; do
for cfg in ${CFGS:-"f32-1" "f32-2" "f32-4" "f16-1" "f16-2" "f16-4"}; do
  pr=${cfg%-*}; t=${cfg#*-}
  EKF_FLUSH_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu --precision $pr --flush-interval $t > gpurun_out/bv_${v}_${pr}_${t}.json 2> gpurun_out/bv.err || { echo "bench $v $cfg failed"; tail -20 gpurun_out/bv.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bv_${v}_${pr}_${t}.json')); print('v$v', '$cfg', round(d['value']), round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, round(d['roofline']['hbm_frac'],3), round(d['roofline']['mfma_frac'],3), d['all_lines_matched'])"
done
done
