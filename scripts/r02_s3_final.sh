# Session-3 final check on the final build: every GPU test, smoke, the driver's bench command (with
# both CPU baselines and the per-scan parity block)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r02_s3_final}
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench2.json 2> $OUT/bench2.err
rc=$?
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
exit $rc
