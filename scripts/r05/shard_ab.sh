#!/bin/bash
# the partitioned instance at a world of one on RCCL: per-scan wall time of the speculative
# protocol for two library builds and the per-line protocol (N = 1024, 24 scans)
set -o pipefail
cd $GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29613 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
out=gpurun_out/r05_shardab; rm -rf $out; mkdir -p $out
for v in base x1024 perline base x1024 perline; do
  mkdir -p $out/$v; lib=slam_ros_amd/lib/libslam_ekf.so; extra=""
  [ $v = x1024 ] && lib=slam_ros_amd/lib/xp_shr1024.so
  [ $v = perline ] && extra="--per-line"
  SLAM_EKF_LIB=$lib timeout -k 10 120 python3 tests/rowshard_gpu_worker.py --out $out/$v --N 1024 --T 4 --scans 24 --precision 1 --backend nccl $extra > $out/$v.log 2>&1 || exit 1
  python3 -c "import numpy as np; d=np.load('$out/$v/rank0.npz'); print('$v', np.median(d['times'])*1e3)" >> $out/summary.txt
  rm -f $out/$v/rank0.npz
done
