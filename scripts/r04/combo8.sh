# fp64 MFMA replay pipelined over (row block, pending step) items (xp_f64p): its identity tests,
# then the fp64 line A/B at T = 8.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04_combo8
mkdir -p $OUT
SLAM_EKF_LIB=slam_ros_amd/lib/xp_f64p.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py -m gpu -v -k "f64 or deferred or speculative or rollback" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "tests failed" > $OUT/status; exit 1; }
SLAM_EKF_LIB=slam_ros_amd/lib/xp_f64q.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py -m gpu -v -k "f64 or deferred or speculative or rollback" --timeout 200 --timeout-method thread > $OUT/pytest_q.log 2>&1 || { echo "q tests failed" > $OUT/status; exit 1; }
VARIANTS="base xp_f64p xp_f64q" STEPS=20 TAG=r04_f64p CONFIGS="--precision f64" bash scripts/r04/ab.sh || exit 5
echo done > $OUT/status
