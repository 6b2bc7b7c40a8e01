# split-bf16 flush timing experiment: bench with the EKF_XP_BF16X6 builds (split, no split, no
# operand reloads), the default build, then the bench-config parity test on the split build
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-xpbf}
mkdir -p $OUT
for v in xp_bf16x6 xp_nosplit xp_noop; do
  SLAM_EKF_LIB=slam_ros_amd/lib/$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_$v.json 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_default.json 2>&1 && \
SLAM_EKF_LIB=slam_ros_amd/lib/xp_bf16x6.so timeout -k 10 300 python -u -m pytest tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k fp32_t8 > $OUT/pytest.log 2>&1
exit 0
