# The split-arithmetic parity tests (bench configs incl. the survey world, split vs exact, association
# identity), then the survey-world and T = 12 profiled lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_combo4
timeout -k 10 600 python -u -m pytest tests/test_bench_config.py tests/test_gpu_parity.py -m gpu -v -k "survey or f16x3 or bf16x6 or speculative or 2x4 or deferred" --timeout 240 --timeout-method thread > gpurun_out/r04_combo4/pytest.log 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json gpurun_out/r04_combo4/ 2>/dev/null
echo "pytest $rc" > gpurun_out/r04_combo4/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
LINES="r04_survey_line|--steps 20 --warmup 5 --world survey;r04_t12|--steps 48 --warmup 20 --flush-interval 12" bash scripts/r04/lines.sh
PROBE_PREC=f64 timeout -k 10 150 python scripts/assoc_probe.py 4096:4 > gpurun_out/r04_combo4/probe_f64.txt 2>&1
PROBE_ARITH=f16x3 PROBE_WORLD=survey timeout -k 10 150 python scripts/assoc_probe.py 4096:20 > gpurun_out/r04_combo4/probe_survey.txt 2>&1
