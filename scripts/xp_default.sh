# default build: parity subset, phase probe, bench (N = 4096 and 1024)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-def}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${KSEL:-spec or deferred or bench_config or trajectory}" > $OUT/pytest.log 2>&1 && \
timeout -k 10 120 python scripts/assoc_probe.py 4096:8 1024:8 > $OUT/probe.txt 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench.json 2>&1 && \
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --capacity 1024 > $OUT/bench1024.json 2>&1
