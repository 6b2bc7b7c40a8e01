# the association kernel's phase timers at the product width (xp_stamps128.so) and the drop-in
set -o pipefail
out=gpurun_out/${TAG}; mkdir -p $out
SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps128.so PROBE_ARITH=f16x3 timeout -k 10 200 python scripts/assoc_probe.py 4096:20 > $out/probe4096.json 2> $out/probe4096.err && \
SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps128.so PROBE_ARITH=f16x3 PROBE_NT=128 timeout -k 10 200 python scripts/assoc_probe.py 1024:12 > $out/probe1024.json 2> $out/probe1024.err && \
TAG=$TAG/dropin bash scripts/r06/dropin.sh
