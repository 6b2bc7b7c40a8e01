# One box: the flush A/B + association timers (measure1.sh), the SURVEY world (survey.sh), then the
# association identity / rollback tests. usage: bash scripts/r04/combo1.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_combo1
bash scripts/r04/measure1.sh; r1=$?
echo "measure1 $r1" > gpurun_out/r04_combo1/status
if [ $r1 -ne 0 ] && [ $r1 -ne 1 ]; then exit $r1; fi
bash scripts/r04/survey.sh; r2=$?
echo "survey $r2" >> gpurun_out/r04_combo1/status
if [ $r2 -gt 1 ]; then exit $r2; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py -m gpu -v -k "speculative or rollback or verdict or singular" --timeout 240 --timeout-method thread > gpurun_out/r04_combo1/pytest_spec.log 2>&1
r3=$?
echo "spec tests $r3" >> gpurun_out/r04_combo1/status
exit $r3
