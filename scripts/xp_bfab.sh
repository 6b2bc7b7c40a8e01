# A/B of split-bf16 flush variants: bf parity tests on the default build, then the bench
# (--arith bf16x6) on the default build and on each $VARIANTS library
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-bfab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bf16x6" > $OUT/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 > $OUT/bench_default.json 2>&1 || exit 1
for v in $VARIANTS; do
  SLAM_EKF_LIB=slam_ros_amd/lib/$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 > $OUT/bench_$v.json 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 > $OUT/bench_default2.json 2>&1
