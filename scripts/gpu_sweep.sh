# bench sweep over schedule × flush variant × flush interval: CFGS="pipe:variant:T[:prec] ..."
# (every run under its own time limit; stops at the first failure)
set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in ${CFGS:-"0:0:4" "1:0:4" "1:6:4" "1:5:4"}; do
  IFS=: read -r pipe var t prec <<< "$cfg"
  prec=${prec:-f32}
  tag="p${pipe}_v${var}_t${t}_${prec}"
  EKF_FLUSH_VARIANT=$var timeout -k 10 150 python bench.py --no-cpu --pipeline $pipe --flush-interval $t \
    --precision $prec --steps ${STEPS:-200} --warmup ${WARMUP:-200} ${EXTRA:-} \
    > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/sweep/$tag.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sweep/$tag.json')); print('$tag', round(d['value']), round(d['ms_per_step'],4), {k: round(x,4) for k,x in d['kernel_ms'].items()}, d['all_lines_matched'])"
done
