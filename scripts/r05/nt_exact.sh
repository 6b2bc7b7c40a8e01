#!/bin/bash
# the narrow association widths in the other flush arithmetics: identity tests, then 48-step lines
set -o pipefail
out=gpurun_out/${TAG:-r05_ntexact}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "narrow" -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
for a in exact bf16x6; do for N in 1024 4096; do for nt in 192 0; do
  timeout -k 10 150 python bench.py --arith $a --capacity $N --scan-threads $nt --steps 48 --warmup 20 --no-cpu > $out/${a}_n${N}_nt${nt}.json 2> $out/${a}_n${N}_nt${nt}.err || exit 1
done; done; done
