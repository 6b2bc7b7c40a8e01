# split-bf16 wave flush with two waves per SIMD (EKF_BF_WAVES=2 build, ring depth 2) vs default
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-w2}
mkdir -p $OUT
for i in 1 2; do
  SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/libslam_ekf_w2.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/w2_$i.json 2>&1 || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/w1_$i.json 2>&1 || exit 1
done
SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/libslam_ekf_w2.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-interval 16 > $OUT/w2_t16.json 2>&1
for f in $OUT/*.json; do python scripts/show_bench.py $f; done > $OUT/summary.txt 2>&1
