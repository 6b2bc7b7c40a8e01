# split-bf16 flush stamps and in-kernel clock (EKF_XP_FLUSH_STAMPS build), T = 8 / 12 / 16, and
# the exact form at T = 8 for comparison
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-bfstamps}
mkdir -p $OUT
export SLAM_EKF_LIB=$GRAFT_REPO_ROOT/slam_ros_amd/lib/libslam_ekf_xp.so
for t in 12 8 16; do
  XP_ARITH=bf16x6 XP_T=$t timeout -k 10 120 python scripts/xp_flush_stamps.py >> $OUT/stamps.jsonl 2> $OUT/err_$t.log || exit 1
done
XP_ARITH=exact XP_T=8 timeout -k 10 120 python scripts/xp_flush_stamps.py >> $OUT/stamps.jsonl 2> $OUT/err_exact.log
