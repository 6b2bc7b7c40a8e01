# full GPU parity suite, then a bench sweep (CFGS); every GPU step time-limited, stop at first failure
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
CFGS="${CFGS:-0:0:8 0:0:6 0:0:4 0:9:4}" bash scripts/gpu_sweep.sh
