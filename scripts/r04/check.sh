# GPU suite (no -x: assertion failures are reported, a crash or timeout ends the call), smoke and
# the driver's bench command with its parity / CPU legs. usage: TAG=<tag> bash scripts/r04/check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r04_check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 ${PYTEST_S:-700} python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc $rc" > $OUT/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { echo "smoke failed" >> $OUT/status; exit 3; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed" >> $OUT/status; exit 4; }
echo "done pytest_rc=$rc" >> $OUT/status
exit $rc
