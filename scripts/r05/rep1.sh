#!/bin/bash
# fp32-MFMA on-read replay: parity subset, survey parity, bench A/B against the plane replay
set -o pipefail
out=gpurun_out/r05_rep1; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_config.py -k "f16x3 and (4096-1-20 or 1024-1-24) or survey" tests/test_gpu_parity.py -k "bf16x6_flush_close or active_flush or speculative_association" > $out/pytest.log 2>&1 &&
for r in 1 2 1 2; do timeout -k 10 150 python bench.py --steps 40 --warmup 20 --no-cpu --mfma-replay $r > $out/bench_rep$r.$RANDOM.json 2>/dev/null || exit 1; done &&
timeout -k 10 600 python -u tests/diag/survey_parity.py f16x3:16,f16x3:20,f16x3:24,bf16x6:16 0 48 > $out/sp.jsonl 2> $out/sp.err
