# A/B of the library built with MFMA accumulators in VGPRs (-mllvm -amdgpu-mfma-vgpr-form,
# slam_ros_amd/lib/libslam_ekf_vgpr.so) against the default build: bit-exactness tests of the
# flush forms with the variant library, then bench lines of both. Every GPU step time-limited.
set -o pipefail
mkdir -p gpurun_out
SLAM_EKF_LIB=$PWD/slam_ros_amd/lib/libslam_ekf_vgpr.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_flush or deferred or speculative" > gpurun_out/gpu_vgpr_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_vgpr_tests.log; exit 1; }
tail -2 gpurun_out/gpu_vgpr_tests.log
for lib in vgpr default; do
  if [ $lib = vgpr ]; then export SLAM_EKF_LIB=$PWD/slam_ros_amd/lib/libslam_ekf_vgpr.so; else unset SLAM_EKF_LIB; fi
  echo "== $lib"
  CFGS="0:0:8:f16 0:0:8 0:83:8" bash scripts/gpu_sweep.sh || exit 1
done
