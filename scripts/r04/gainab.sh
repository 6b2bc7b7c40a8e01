# A/B of the speculative gain-row corrections (xp_pairs: EKF_GAIN_FIXQ=0) plus the association
# identity / rollback tests and the phase timers of the product build.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_gain
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py -m gpu -v -k "speculative or rollback or verdict or singular or deferred" --timeout 240 --timeout-method thread > gpurun_out/r04_gain/pytest.log 2>&1
rc=$?
echo "pytest $rc" > gpurun_out/r04_gain/status
if [ $rc -ne 0 ]; then exit $rc; fi
STEPS=20 TAG=r04_gain VARIANTS="base xp_pairs" CONFIGS="--arith f16x3;--arith f16x3 --capacity 1024" bash scripts/r04/ab.sh && \
PROBE_ARITH=f16x3 timeout -k 10 120 python scripts/assoc_probe.py 4096:20 1024:20 > gpurun_out/r04_gain/probe.txt 2>&1
