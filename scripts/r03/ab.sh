# A/B timing of library variants on one box: association stamps (4096:12) and the bench line, each
# variant twice in alternating order. LIBS="base xp_a xp_b ..." (base = libslam_ekf.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_ab}
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for v in ${LIBS:-base}; do
    if [ "$v" = base ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/$v.so; fi
    SLAM_EKF_LIB=$lib timeout -k 10 120 python scripts/assoc_probe.py ${PROBE_CFG:-4096:12} > gpurun_out/$TAG/probe_${v}_$rep.txt 2>&1 || exit 1
    SLAM_EKF_LIB=$lib timeout -k 10 120 python bench.py --steps 48 --warmup 200 --no-cpu ${BENCH_ARGS} > gpurun_out/$TAG/bench_${v}_$rep.json 2>&1 || exit 1
  done
done
echo done > gpurun_out/$TAG/status
