# A/B timing builds: bash scripts/build_ab.sh NAME KERNELS.hip → slam_ros_amd/lib/xp_NAME.so (the
# given kernel source with this tree's API source; selected at run time by SLAM_EKF_LIB)
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
mkdir -p $T/include $T/p/csrc
cp include/slam_ekf.h $T/include/
cp slam_ros_amd/csrc/*.h slam_ros_amd/csrc/ekf_api.hip $T/p/csrc/
cp "$2" $T/p/csrc/ekf_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -mllvm -amdgpu-mfma-vgpr-form \
  -o slam_ros_amd/lib/xp_$1.so $T/p/csrc/ekf_kernels.hip $T/p/csrc/ekf_api.hip
rm -rf $T
