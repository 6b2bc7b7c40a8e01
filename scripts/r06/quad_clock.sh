# In-kernel clock of the quad flush's timing variants (xp_qC*.so, -DEKF_Q_CLOCK builds)
# usage: TAG=<tag> VARIANTS="qC qCNT ..." bash scripts/r06/quad_clock.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_qclock}; mkdir -p $out
for v in $VARIANTS; do
  SLAM_EKF_LIB=slam_ros_amd/lib/xp_$v.so timeout -k 10 120 python scripts/r06/quad_clock.py > $out/$v.json 2> $out/$v.err || exit 1
  SLAM_EKF_LIB=slam_ros_amd/lib/xp_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $out/${v}_bench.json 2> $out/${v}_bench.err || exit 1
done
