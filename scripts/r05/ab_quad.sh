#!/bin/bash
# the split-fp16 quad flush (EKF_OPT_FLUSH_FORM = 44, scripts/xp/f16_quad_flush.patch applied): its identity
# test against the 2 x 2 wave form,
# then bench lines of both forms alternating (quad4: exchanges of four steps, xp_q4.so) (48 timed steps; N = 4096 T = 20 and 12, fp16 storage)
set -o pipefail
out=gpurun_out/r05_abquad; rm -rf $out; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "quad or 2x4" -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
for rep in 1 2; do
  for v in wave quad quad4; do
    ff=44; [ $v = wave ] && ff=0
    lib=slam_ros_amd/lib/libslam_ekf.so; [ $v = quad4 ] && lib=slam_ros_amd/lib/xp_q4.so
    for cfg in "T20|--flush-interval 20" "T12|--flush-interval 12" "f16|--precision f16"; do
      tag="${cfg%%|*}"; args="${cfg#*|}"
      SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps 48 --warmup 20 --no-cpu --flush-form $ff $args > $out/${v}_${tag}_$rep.json 2> $out/${v}_${tag}_$rep.err || exit 1
      python -c "import json; d=json.load(open('$out/${v}_${tag}_$rep.json')); print('$v $tag rep $rep', round(d['value']), 'flush ms', round(d['kernel_ms']['flush'],4), 'scan ms', round(d['kernel_ms']['scan'],4), d['roofline']['kernel'])" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
