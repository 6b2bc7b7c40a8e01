set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bisect
for v in v_k6; do
  if [ $v = default ]; then unset SLAM_EKF_LIB; else export SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/lib_$v.so; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "deferred" > gpurun_out/bisect/$v.log 2>&1
  echo "$v rc=$?" >> gpurun_out/bisect/summary.txt
done
exit 0
