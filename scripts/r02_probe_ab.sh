cd $GRAFT_REPO_ROOT
for v in default p_nolds p_noload p_both; do
  if [ $v = default ]; then unset SLAM_EKF_LIB; else export SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/lib_$v.so; fi
  echo "== $v" >> gpurun_out/probe_ab.txt
  timeout -k 10 100 python scripts/assoc_probe.py 4096:8 >> gpurun_out/probe_ab.txt 2>&1 || exit 1
done
