#!/bin/bash
# the partitioned instance at a world of one on RCCL: kernel trace of the speculative and the
# per-line protocols (N = 1024, 24 scans each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
out=gpurun_out/r05_shardprof; rm -rf $out; mkdir -p $out/spec $out/perline
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/kt_spec -o run --output-format csv -- python3 tests/rowshard_gpu_worker.py --out $out/spec --N 1024 --T 4 --scans 24 --precision 1 --backend nccl > $out/spec.log 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/kt_perline -o run --output-format csv -- python3 tests/rowshard_gpu_worker.py --out $out/perline --N 1024 --T 4 --scans 24 --precision 1 --backend nccl --per-line > $out/perline.log 2>&1
python3 -c "import numpy as np, json; [json.dump({'times': np.load('$out/%s/rank0.npz' % m)['times'].tolist(), 'spec_runs': np.load('$out/%s/rank0.npz' % m)['spec_runs'].tolist()}, open('$out/%s.json' % m, 'w')) for m in ('spec', 'perline')]"; rm -f $out/*/rank0.npz; find $out -name "*kernel_trace.csv" -delete; find $out -name "*agent_info.csv" -delete; du -sh $out
