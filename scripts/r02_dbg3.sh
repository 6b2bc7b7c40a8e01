cd $GRAFT_REPO_ROOT
for v in default; do
  if [ $v = default ]; then unset SLAM_EKF_LIB; else export SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/lib_$v.so; fi
  echo "== $v" >> gpurun_out/dbg3.txt
  timeout -k 10 100 python scripts/dbg_deferred3.py >> gpurun_out/dbg3.txt 2>&1 || exit 1
done
