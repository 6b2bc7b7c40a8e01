# The GPU suite on the shared-owned-row replay build, the fp64 line A/B (4 vs 2 columns per pass
# over the pending steps), the fp64 association probe, then the SURVEY-world path histogram.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04_combo5
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest $rc" > $OUT/status
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS="base xp_pb2" STEPS=20 TAG=r04_pb64 CONFIGS="--precision f64" bash scripts/r04/ab.sh || exit 5
PROBE_PREC=f64 timeout -k 10 150 python scripts/assoc_probe.py 4096:4 > $OUT/probe_f64.txt 2>&1 || exit 6
timeout -k 10 300 python scripts/r04/survey_diag.py 20 200 60 > $OUT/sdiag.txt 2>&1 || exit 7
exit $rc
