# Wave-flush A/B: its bit-exactness tests (incl. the fp32 opt-in variant 83), then bench lines.
# Every GPU step under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_flush or deferred" > gpurun_out/gpu_wave_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_wave_tests.log; exit 1; }
tail -2 gpurun_out/gpu_wave_tests.log
EKF_WAVE_TEST_VARIANT=83 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_flush" > gpurun_out/gpu_wave83_tests.log 2>&1 || { echo "pytest v83 failed"; tail -40 gpurun_out/gpu_wave83_tests.log; exit 1; }
tail -2 gpurun_out/gpu_wave83_tests.log
CFGS="${CFGS:-0:0:8:f16 0:83:8 0:0:8 0:0:6:f16}" bash scripts/gpu_sweep.sh
