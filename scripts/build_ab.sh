# A/B timing builds: bash scripts/build_ab.sh NAME KERNELS.hip → slam_ros_amd/lib/xp_NAME.so (the
# given kernel source with this tree's API source and headers; the library's compilation units in
# parallel; selected at run time by SLAM_EKF_LIB)
set -e
cd "$(dirname "$0")/.."
T=$(mktemp -d)
mkdir -p $T/include $T/p/csrc
cp include/slam_ekf.h $T/include/
cp slam_ros_amd/csrc/*.h slam_ros_amd/csrc/ekf_api.hip $T/p/csrc/
cp "$2" $T/p/csrc/ekf_kernels.hip
python3 -c "import sys; sys.path.insert(0, '.'); from slam_ros_amd import build as b; b.build_variant('slam_ros_amd/lib/xp_$1.so', [], csrc='$T/p/csrc')"
rm -rf $T
