#!/bin/bash
# A/B: the split flush's prologue order (loop-head wait without draining the stores) vs the build
# before it (slam_ros_amd/lib/xp_base.so), alternating, 48 timed steps
set -o pipefail
out=gpurun_out/r05_abflush; mkdir -p $out
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/xp_base.so; fi
    for T in 20 12; do
      SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps 48 --warmup 20 --no-cpu --flush-interval $T > $out/${v}_T${T}_$rep.json 2> $out/${v}_T${T}_$rep.err || exit 1
    done
  done
done
