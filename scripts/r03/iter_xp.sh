# iteration (tests, stamps, bench) then the bench on each $VARIANTS library (timing experiments)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_iter}
bash scripts/r03/iter.sh || exit 1
for v in $VARIANTS; do
  SLAM_EKF_LIB=slam_ros_amd/lib/$v.so timeout -k 10 120 python bench.py --steps 48 --warmup 200 --no-cpu > gpurun_out/$TAG/bench_$v.json 2>&1 || exit 1
done
timeout -k 10 120 env EKF_FLUSH_VARIANT=24 python bench.py --steps 48 --warmup 200 --no-cpu > gpurun_out/$TAG/bench_2x4.json 2>&1
