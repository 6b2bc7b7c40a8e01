# wave-flush A/B: parity (forced variant 8) then a bench sweep; every GPU step time-limited
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "wave_flush or deferred" > gpurun_out/wave_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/wave_tests.log; exit 1; }
tail -2 gpurun_out/wave_tests.log
CFGS="${CFGS:-0:8:4 0:8:6 0:8:8 0:0:4}" bash scripts/gpu_sweep.sh
