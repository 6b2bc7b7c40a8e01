# fp64 flush A/B: the full GPU parity suite on the current build, then fp64 bench lines of the
# current build and of slam_ros_amd/lib/libslam_ekf_prev.so. Every GPU step time-limited.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for lib in new prev; do
  if [ $lib = prev ]; then export SLAM_EKF_LIB=$PWD/slam_ros_amd/lib/libslam_ekf_prev.so; else unset SLAM_EKF_LIB; fi
  echo "== $lib"
  CFGS="0:0:4:f64 0:0:8:f64" bash scripts/gpu_sweep.sh || exit 1
done
