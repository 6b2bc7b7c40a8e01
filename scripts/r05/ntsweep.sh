#!/bin/bash
# landmarks per association workgroup (EKF_OPT_SCAN_THREADS): identity test, then 48-step bench
# lines per capacity and width (split-fp16, the bench's T per capacity)
set -o pipefail
out=gpurun_out/${TAG:-r05_ntsweep}; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "narrow or hot_scan" -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
for N in ${NS:-256 1024 4096}; do for nt in 192 128 64; do
  timeout -k 10 120 python bench.py --capacity $N --scan-threads $nt --steps 48 --warmup 20 --no-cpu > $out/n${N}_nt${nt}.json 2> $out/n${N}_nt${nt}.err || exit 1
done; done
