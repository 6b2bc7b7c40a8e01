# phase timers of two stamp builds at the product width, alternating (xp_stamps128_base.so, xp_stamps128.so)
set -o pipefail
out=gpurun_out/${TAG}; mkdir -p $out
for r in 1 2; do for v in stamps128_base stamps128; do
  SLAM_EKF_LIB=slam_ros_amd/lib/xp_$v.so PROBE_ARITH=f16x3 timeout -k 10 200 python scripts/assoc_probe.py 4096:20 > $out/${v}_$r.json 2> $out/${v}_$r.err || exit 1
done; done
