#!/bin/bash
# the partitioned instance: GPU tests, then the per-scan wall time at a world of one on RCCL of the
# Python-driven protocol (rowshard_gpu.py phases + torch.distributed collectives) and of the native
# call (ekf_shard_localize on the library's own communicator), N = 1024 / 4096, fp32 and fp64
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/r05_shardab3; rm -rf $out; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_rowshard_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29619 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for rep in 1 2; do
  for v in py native; do
    for cfg in "1024|1" "4096|1" "1024|0"; do
      N="${cfg%%|*}"; prec="${cfg#*|}"; extra=""; [ $v = native ] && extra="--native"
      d=$out/$v${N}p$prec; mkdir -p $d
      timeout -k 10 120 python3 tests/rowshard_gpu_worker.py --out $d --N $N --T 4 --scans 24 --precision $prec --backend nccl $extra > $d.log 2>&1 || exit 1
      python3 -c "import numpy as np; d=np.load('$d/rank0.npz'); t=d['times'][4:]; print('$v N=$N prec=$prec rep $rep median', round(float(np.median(t))*1e3, 4), 'ms min', round(float(t.min())*1e3, 4))" >> $out/summary.txt
      rm -f $d/rank0.npz
    done
  done
done
cat $out/summary.txt
