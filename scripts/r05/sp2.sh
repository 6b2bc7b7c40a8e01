#!/bin/bash
# survey world: per-scan y/pose re-sync (SP_PER_SCAN=1), fp32 MFMA replay (1) vs plane replay (2), exact
set -o pipefail
out=gpurun_out/r05_sp2; mkdir -p $out
export SP_PER_SCAN=1
timeout -k 10 600 python -u tests/diag/survey_parity.py f16x3:20,f16x3:24,f16x3:20:mfma_replay=2,f16x3:24:mfma_replay=2,exact:16,bf16x6:16 0 48 > $out/pre0.jsonl 2> $out/pre0.err &&
timeout -k 10 600 python -u tests/diag/survey_parity.py f16x3:20,f16x3:20:mfma_replay=2,exact:16 200 48 > $out/pre200.jsonl 2> $out/pre200.err
