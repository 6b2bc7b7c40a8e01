#!/bin/bash
# A/B: U rows not stored for symmetric operands (readers scale V) vs the build before
# (slam_ros_amd/lib/xp_base.so), alternating, 48 timed steps
set -o pipefail
out=gpurun_out/${TAG:-r05_abusym}; mkdir -p $out
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = new ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/xp_base.so; fi
    SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps 48 --warmup 20 --no-cpu --scan-threads 128 > $out/${v}_n4096_$rep.json 2> $out/${v}_n4096_$rep.err || exit 1
    SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --capacity 1024 --steps 48 --warmup 20 --no-cpu > $out/${v}_n1024_$rep.json 2> $out/${v}_n1024_$rep.err || exit 1
  done
done
