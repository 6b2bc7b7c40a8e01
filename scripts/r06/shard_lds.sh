# the partitioned run with each landmark's record, history rows and flags in LDS
# (explicit slots, bounds-checked): the rowshard GPU tests on a build that prints any landmark
# outside its workgroup's slots (EKF_SHR_BOUNDS), once, in a fresh directory; then the one-call
# scan's wall time, this build against the previous one (xp_shbase.so), world of one on RCCL.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_shardlds}; mkdir -p $out
SLAM_EKF_LIB=slam_ros_amd/lib/xp_shbounds.so timeout -k 10 400 python -u -m pytest tests/test_rowshard_gpu.py -x -v -s --timeout 120 --timeout-method thread > $out/pytest_bounds.log 2>&1 || exit 1
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29619 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for rep in 1 2; do
  for lib in product shbase; do
    for cfg in "1024|1" "4096|1" "1024|0"; do
      N="${cfg%%|*}"; prec="${cfg#*|}"
      d=$out/$lib${N}p$prec; mkdir -p $d
      if [ $lib = product ]; then L=slam_ros_amd/lib/libslam_ekf.so; else L=slam_ros_amd/lib/xp_$lib.so; fi
      SLAM_EKF_LIB=$L timeout -k 10 120 python3 tests/rowshard_gpu_worker.py --out $d --N $N --T 4 --scans 24 --precision $prec --backend nccl --native > $d.log 2>&1 || exit 1
      python3 -c "import numpy as np; d=np.load('$d/rank0.npz'); t=d['times'][4:]; print('$lib N=$N prec=$prec rep $rep median', round(float(np.median(t))*1e3, 4), 'ms min', round(float(t.min())*1e3, 4))" >> $out/summary.txt
      rm -f $d/rank0.npz
    done
  done
done
cat $out/summary.txt
