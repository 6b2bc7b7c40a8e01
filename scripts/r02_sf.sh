# staged replay without the per-block scheduling barrier (EKF_XP_STAGED_FREE build) vs default:
# speculative-path identity tests on the variant, then bench at T = 12 and 16
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-sf}
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/slam_ros_amd/lib/libslam_ekf_sf.so
SLAM_EKF_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "speculative or deferred" > $OUT/pytest.log 2>&1 || exit 1
for i in 1 2; do
  SLAM_EKF_LIB=$V timeout -k 10 120 python bench.py --steps 48 --warmup 12 --no-cpu > $OUT/sf_$i.json 2>&1 || exit 1
  timeout -k 10 120 python bench.py --steps 48 --warmup 12 --no-cpu > $OUT/base_$i.json 2>&1 || exit 1
done
for f in $OUT/*.json; do python scripts/show_bench.py $f; done > $OUT/summary.txt 2>&1
