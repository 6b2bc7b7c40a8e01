# Round 6 start: the driver's bench command on the shipped library, and the association kernel's
# phase timers at the product width (xp_stamps128.so, scripts/r06/stamp_build.sh)
set -o pipefail
out=gpurun_out/${TAG:-r06_base}; mkdir -p $out
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err && \
SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps128.so PROBE_ARITH=f16x3 timeout -k 10 200 python scripts/assoc_probe.py 4096:20 > $out/probe4096.json 2> $out/probe4096.err && \
SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps128.so PROBE_ARITH=f16x3 PROBE_NT=128 timeout -k 10 200 python scripts/assoc_probe.py 1024:12 > $out/probe1024.json 2> $out/probe1024.err
