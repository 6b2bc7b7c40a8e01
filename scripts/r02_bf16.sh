# split-bf16 flush with up to 16 steps per group: parity tests, then bench at T = 8 and 16
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-bf16}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${KSEL:-bf16x6 or deferred or wave_flush or speculative or bench_config_fp32}" > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 > $OUT/bench_bf8.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 --flush-interval 16 > $OUT/bench_bf16.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 --flush-interval 12 > $OUT/bench_bf12.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_exact8.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --arith bf16x6 --flush-interval 16 --capacity 1024 > $OUT/bench_bf16_1024.json 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
exit $rc
