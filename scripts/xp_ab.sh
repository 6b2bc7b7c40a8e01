# A/B of a variant library (SLAM_EKF_LIB=$LIB): parity subset, phase probe and bench, then the
# same probe and bench on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
SLAM_EKF_LIB=$LIB timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${KSEL:-spec or deferred or bench_config or trajectory}" > $OUT/pytest.log 2>&1 && \
SLAM_EKF_LIB=$LIB timeout -k 10 120 python scripts/assoc_probe.py 4096:8 1024:8 > $OUT/probe_b.txt 2>&1 && \
SLAM_EKF_LIB=$LIB timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_b.json 2>&1 && \
SLAM_EKF_LIB=$LIB timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --capacity 1024 > $OUT/bench_b1024.json 2>&1 && \
timeout -k 10 120 python scripts/assoc_probe.py 4096:8 1024:8 > $OUT/probe_a.txt 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_a.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --capacity 1024 > $OUT/bench_a1024.json 2>&1
