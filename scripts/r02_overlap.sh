# association kernels overlapping the previous group's flush (pipeline = 1, G > 1): the
# EKF_PIPE_OVERLAP hook lifts the serialisation; the variant build caps the flush at 256
# registers per wave with one workgroup per CU (room for an association workgroup beside it)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-overlap}
mkdir -p $OUT
V=$GRAFT_REPO_ROOT/slam_ros_amd/lib/libslam_ekf_ov.so
SLAM_EKF_LIB=$V timeout -k 10 120 python bench.py --steps 40 --warmup 8 --no-cpu --flush-interval 8 > $OUT/ov_base_t8.json 2>&1 || exit 1
SLAM_EKF_LIB=$V EKF_PIPE_OVERLAP=1 timeout -k 10 120 python bench.py --steps 40 --warmup 8 --no-cpu --flush-interval 8 --pipeline 1 > $OUT/ov_pipe_t8.json 2>&1 || exit 1
EKF_PIPE_OVERLAP=1 timeout -k 10 120 python bench.py --steps 40 --warmup 8 --no-cpu --flush-interval 8 --pipeline 1 > $OUT/main_pipe_t8.json 2>&1 || exit 1
SLAM_EKF_LIB=$V EKF_PIPE_OVERLAP=1 timeout -k 10 120 python bench.py --steps 48 --warmup 12 --no-cpu --flush-interval 12 --pipeline 1 > $OUT/ov_pipe_t12.json 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 48 --warmup 12 --no-cpu > $OUT/main_seq_t12.json 2>&1
for f in $OUT/*.json; do python scripts/show_bench.py $f; grep -o '"all_lines_matched": [a-z]*' $f; done > $OUT/summary.txt 2>&1
