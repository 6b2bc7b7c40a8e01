#!/bin/bash
# survey-world parity diagnosis (tests/diag/survey_parity.py), from init and after a 200-scan pre-roll
set -o pipefail
out=gpurun_out/r05_sp; mkdir -p $out
timeout -k 10 500 python -u tests/diag/survey_parity.py ${1:-exact:16,f16x3:16,f16x3:20,bf16x6:16} 0 48 > $out/pre0.jsonl 2> $out/pre0.err &&
timeout -k 10 600 python -u tests/diag/survey_parity.py ${1:-exact:16,f16x3:16,f16x3:20,bf16x6:16} 200 48 > $out/pre200.jsonl 2> $out/pre200.err
