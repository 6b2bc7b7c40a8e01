# Round 2, session 3 check on the rebuilt library: every GPU test, smoke, the driver's bench command
# (with both CPU baselines) and the PMC profile of the default bench line (bf16x6, T = 12)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r02_s3}
mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 && \
timeout -k 10 60 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err && \
TAG=r02_bf16_final bash scripts/pmc_profile.sh --steps 20 --warmup 5
rc=$?
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
exit $rc
