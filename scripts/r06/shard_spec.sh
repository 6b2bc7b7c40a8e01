# the partitioned run in the association kernel's form (shard_spec_kernel: one
# verdict exchange per run instead of one per line): the rowshard GPU tests once, in a fresh
# directory, then the one-call scan's wall time against the per-line-exchange build (xp_shrun.so,
# EKF_SHARD_SPEC=0), world of one on RCCL, and a kernel-trace profile of the N=1024 fp32 case.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_shardspec}; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests/test_rowshard_gpu.py -x -v -s --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29619 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
for rep in 1 2; do
  for lib in ${LIBS:-product shrun}; do
    for cfg in "1024|1" "4096|1" "1024|0" "16384|1"; do
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
cd /tmp && export TMPDIR=/tmp
d=$GRAFT_REPO_ROOT/$out/prof1024; mkdir -p $d
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/rp -o shard --output-format csv -- python3 $GRAFT_REPO_ROOT/tests/rowshard_gpu_worker.py --out $d --N 1024 --T 4 --scans 24 --precision 1 --backend nccl --native > $GRAFT_REPO_ROOT/$out/rp.log 2>&1 || exit 1
rm -f $d/rank0.npz
