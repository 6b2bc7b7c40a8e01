# Unconditional next-tile loads (no wait-count drain at the wave-tile loop head): fp64 flush A/B
# (xp_t64) and split-fp16 flush A/B (xp_t16), each variant's bit-identity tests first.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04_combo7
mkdir -p $OUT
SLAM_EKF_LIB=slam_ros_amd/lib/xp_t64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "f64_wave or f64_mfma or deferred" --timeout 200 --timeout-method thread > $OUT/pytest_t64.log 2>&1 || { echo "t64 tests failed" > $OUT/status; exit 1; }
SLAM_EKF_LIB=slam_ros_amd/lib/xp_t16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "2x4 or deferred" --timeout 200 --timeout-method thread > $OUT/pytest_t16.log 2>&1 || { echo "t16 tests failed" > $OUT/status; exit 1; }
VARIANTS="base xp_t64" STEPS=20 TAG=r04_t64 CONFIGS="--precision f64" bash scripts/r04/ab.sh || exit 5
VARIANTS="base xp_t16" STEPS=20 TAG=r04_t16 CONFIGS="--arith f16x3;--arith f16x3 --flush-interval 12" bash scripts/r04/ab.sh || exit 6
echo done > $OUT/status
