#!/bin/bash
# A/B of the association width at larger capacities: alternating runs, 48 timed steps
set -o pipefail
out=gpurun_out/${TAG:-r05_ntab}; mkdir -p $out
for r in 1 2 3; do for N in 4096 2048; do for nt in 192 128 64; do
  timeout -k 10 120 python bench.py --capacity $N --scan-threads $nt --steps 48 --warmup 20 --no-cpu > $out/n${N}_nt${nt}_r$r.json 2> $out/n${N}_nt${nt}_r$r.err || exit 1
done; done; done
