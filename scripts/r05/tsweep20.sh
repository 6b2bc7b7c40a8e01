#!/bin/bash
# flush interval per capacity at the driver's window (20 timed steps, 5 warm-up), two runs each
set -o pipefail
out=gpurun_out/${TAG:-r05_tsweep20}; mkdir -p $out
for r in 1 2; do
for N in 256 1024; do for T in ${TS:-2 4 6 8 12}; do
  timeout -k 10 120 python bench.py --capacity $N --flush-interval $T --steps 20 --warmup 5 --no-cpu > $out/n${N}_t${T}_$r.json 2> $out/n${N}_t${T}_$r.err || exit 1
done; done; done
