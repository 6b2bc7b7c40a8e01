#!/bin/bash
# the partitioned instance at a world of one on RCCL: kernel trace of the speculative protocol
# (N = 1024, 24 scans; cooperating-workgroup run; NATIVE=1: the one-call path)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=29617 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
out=gpurun_out/r05_shardprof2; rm -rf $out; mkdir -p $out/spec
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/kt_spec -o run --output-format csv -- python3 tests/rowshard_gpu_worker.py --out $out/spec --N 1024 --T 4 --scans 24 --precision 1 --backend nccl ${NATIVE:+--native} > $out/spec.log 2>&1
rc=$?
rm -f $out/spec/rank0.npz; find $out -name "*agent_info.csv" -delete
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open('gpurun_out/r05_shardprof2/kt_spec/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# the last 10 scans: every dispatch between consecutive shard_run_kernel launches
runs = [k for k, r in enumerate(rows) if 'shard_run_kernel' in r['Kernel_Name']]
for a, b in zip(runs[-4:-1], runs[-3:]):
    t0 = int(rows[a]['Start_Timestamp'])
    for r in rows[a:b]:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:7.1f} us  {r['Kernel_Name'][:70]}")
    print('---')
PY
find $out -name "*kernel_trace.csv" -delete
exit $rc
