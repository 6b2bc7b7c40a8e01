#!/bin/bash
# flush interval per capacity: 20- and 48-step windows
set -o pipefail
out=gpurun_out/${TAG:-r05_tsweep2}; mkdir -p $out
for r in 1 2; do
for spec in "256 4" "256 8" "256 16" "1024 8" "1024 12" "1024 16" "1024 20"; do
  set -- $spec; N=$1; T=$2
  for K in 20 48; do
    timeout -k 10 120 python bench.py --capacity $N --flush-interval $T --steps $K --warmup 5 --no-cpu > $out/n${N}_t${T}_k${K}_$r.json 2> $out/n${N}_t${T}_k${K}_$r.err || exit 1
  done
done; done
