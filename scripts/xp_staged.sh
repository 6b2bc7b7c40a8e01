# staged-replay timing experiment: default build vs no per-step row loads vs no FMA chains
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/xp
timeout -k 10 120 python scripts/assoc_probe.py 4096:8 > gpurun_out/xp/base.txt 2>&1 && \
PROBE_NOASSERT=1 SLAM_EKF_LIB=slam_ros_amd/lib/xp_noload.so timeout -k 10 120 python scripts/assoc_probe.py 4096:8 > gpurun_out/xp/noload.txt 2>&1 && \
PROBE_NOASSERT=1 SLAM_EKF_LIB=slam_ros_amd/lib/xp_nofma.so timeout -k 10 120 python scripts/assoc_probe.py 4096:8 > gpurun_out/xp/nofma.txt 2>&1
