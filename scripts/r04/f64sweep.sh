# fp64 wave flush with the operand ring (groups of up to 8 steps): its bit-identity tests, then the
# fp64 bench line at T = 4, 6, 8 (driver's 20 steps and 48). usage: bash scripts/r04/f64sweep.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_f64sweep
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "f64_wave or deferred" --timeout 200 --timeout-method thread > gpurun_out/r04_f64sweep/pytest.log 2>&1
rc=$?
echo "pytest $rc" > gpurun_out/r04_f64sweep/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
C="--precision f64 --flush-interval 4;--precision f64 --flush-interval 6;--precision f64 --flush-interval 8"
STEPS=20 TAG=r04_f64sweep20 CONFIGS="$C" bash scripts/r04/ab.sh && \
STEPS=48 TAG=r04_f64sweep48 CONFIGS="$C" bash scripts/r04/ab.sh
