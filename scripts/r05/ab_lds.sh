#!/bin/bash
# timing probe (results invalid): the split-fp16 flush with half of each wave's operand planes
# loaded from global memory and the other half read from a partner wave's LDS slot, one barrier per
# four steps (slam_ros_amd/lib/xp_lds.so, built from a patched copy) against the product build,
# alternating, 48 timed steps
set -o pipefail
out=gpurun_out/r05_ablds; mkdir -p $out
for rep in 1 2; do
  for v in base lds; do
    lib=slam_ros_amd/lib/libslam_ekf.so; [ $v = lds ] && lib=slam_ros_amd/lib/xp_lds.so
    for T in 20 12; do
      SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps 48 --warmup 20 --no-cpu --flush-interval $T > $out/${v}_T${T}_$rep.json 2> $out/${v}_T${T}_$rep.err || exit 1
      python -c "import json,sys; d=json.load(open('$out/${v}_T${T}_$rep.json')); print('$v T=$T rep $rep', round(d['value']), 'flush ms', round(d['kernel_ms']['flush'],4), 'scan ms', round(d['kernel_ms']['scan'],4))" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
