#!/bin/bash
# L1 / L2 counters of the bench's kernels (one pass each), N = 4096 default line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r05_l1l2; rm -rf $out; mkdir -p $out
timeout -s KILL 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $GRAFT_REPO_ROOT/$out/p1 -o run --output-format csv -- python3 bench.py --no-cpu --steps 20 --warmup 5 > $out/p1.log 2>&1
