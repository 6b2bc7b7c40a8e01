#!/bin/bash
# round-5 parity additions: survey-world parity (init, steady), RCCL world-1 broadcast, partitioned
# instance vs the oracle, pipelined active flush; bench A/B of the replay forms
set -o pipefail
out=gpurun_out/r05_check2; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  "tests/test_bench_config.py::test_survey_world_parity_from_init" "tests/test_bench_config.py::test_survey_world_parity_steady_state" \
  tests/test_bench_multirank.py::test_rccl_grouped_broadcast_world1 tests/test_rowshard_gpu.py \
  tests/test_gpu_parity.py::test_active_flush_pipelined_reset_and_upload > $out/pytest.log 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json $out/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
for r in 1 2 1 2; do timeout -k 10 150 python bench.py --steps 40 --warmup 20 --no-cpu --mfma-replay $r > $out/bench_rep$r.$RANDOM.json 2>/dev/null || exit 1; done
