# GPU parity suite, fp16 (config 5) and fp32 bench lines, then the default bench with its
# rocprofv3 kernel-trace stats and FETCH/WRITE/SQ passes. Every GPU step runs under its own time
# limit and the steps are chained, so the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
CFGS="${CFGS:-0:0:8:f16 0:0:8}" bash scripts/gpu_sweep.sh || exit 1
bash scripts/gpu_bench_profile.sh
rc=$?
cat gpurun_out/bench.json
exit $rc
