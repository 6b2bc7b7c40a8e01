# SURVEY §8d world: the association-path histogram (tests/test_bench_config.py::test_survey_world_association
# records it) and the bench line in that world. usage: bash scripts/r04/survey.sh → gpurun_out/r04_survey/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r04_survey}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_bench_config.py -m gpu -v -k survey --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json $OUT/ 2>/dev/null
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc" > $OUT/status; exit $rc; fi
timeout -k 10 200 python bench.py --steps 48 --warmup 24 --no-cpu --world survey ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc2=$?
echo "pytest $rc bench $rc2" > $OUT/status
exit $rc2
