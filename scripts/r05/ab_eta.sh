#!/bin/bash
# A/B in SURVEY §8d's world: the gate's storage-precision bounds (product) vs none (xp_noeta.so)
set -o pipefail
out=gpurun_out/${TAG:-r05_abeta}; mkdir -p $out
for rep in 1 2; do for v in new noeta; do
  if [ $v = new ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/xp_noeta.so; fi
  for T in 8 12; do
    SLAM_EKF_LIB=$lib timeout -k 10 200 python bench.py --world survey --flush-interval $T --steps 48 --warmup 20 --no-cpu > $out/${v}_T${T}_$rep.json 2> $out/${v}_T${T}_$rep.err || exit 1
  done
done; done
