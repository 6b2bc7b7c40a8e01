# Active-map split flush (EKF_OPT_ACTIVE_FLUSH): its identity tests and the split-arithmetic /
# survey / rollback parity tests on the new build, then A/B against the previous build (xp_old)
# on the bench default and the SURVEY world, and the new build's survey line with the option off.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04_combo9
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config.py tests/test_rollback.py -m gpu -v -k "active_flush" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest $rc" > $OUT/status
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="base xp_old" STEPS=20 TAG=r04_active CONFIGS="--arith f16x3;--world survey" bash scripts/r04/ab.sh || exit 5
echo done >> $OUT/status
