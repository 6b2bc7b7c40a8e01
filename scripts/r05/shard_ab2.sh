#!/bin/bash
# the partitioned instance: GPU tests on this build, then the per-scan wall time of the speculative
# protocol at a world of one on RCCL for the previous build (slam_ros_amd/lib/xp_base.so: the run on
# one 1024-thread workgroup) and this one (cooperating 128-landmark workgroups; shr64: 64), N = 1024 / 4096
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/r05_shardab2; rm -rf $out; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_rowshard_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29615 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for rep in 1 2; do
  for v in base new shr64; do
    for N in 1024 4096; do
      mkdir -p $out/$v$N; lib=slam_ros_amd/lib/libslam_ekf.so
      [ $v = base ] && lib=slam_ros_amd/lib/xp_base.so
      [ $v = shr64 ] && lib=slam_ros_amd/lib/xp_shr64.so
      SLAM_EKF_LIB=$lib timeout -k 10 120 python3 tests/rowshard_gpu_worker.py --out $out/$v$N --N $N --T 4 --scans 24 --precision 1 --backend nccl > $out/$v$N.log 2>&1 || exit 1
      python3 -c "import numpy as np; d=np.load('$out/$v$N/rank0.npz'); print('$v N=$N rep $rep', round(np.median(d['times'])*1e3, 4), 'ms', 'runs', sorted(set(d['spec_runs'].tolist())))" >> $out/summary.txt
      rm -f $out/$v$N/rank0.npz
    done
  done
done
cat $out/summary.txt
