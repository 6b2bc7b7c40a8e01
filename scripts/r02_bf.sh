# split-bf16 flush (EKF_ARITH_BF16X6): its parity tests, the exact-path schedule tests, then the
# bench in both arithmetics
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-bf}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${KSEL:-bf16x6 or deferred or wave_flush}" > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 > $OUT/bench_bf.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_exact.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 --capacity 1024 > $OUT/bench_bf1024.json 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
exit $rc
