#!/bin/bash
# flush interval per capacity: N = 256 / 1024, split-fp16, 48 timed steps
set -o pipefail
out=gpurun_out/r05_tsweep; mkdir -p $out
for N in 256 1024; do for T in 4 6 8 12 16 20; do
  timeout -k 10 120 python bench.py --capacity $N --flush-interval $T --steps 48 --warmup 20 --no-cpu > $out/n${N}_t${T}.json 2> $out/n${N}_t${T}.err || exit 1
done; done
