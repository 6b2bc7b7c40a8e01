# The one-call partitioned scan at N = 32768 (MAX_CAPACITY; shard_spec_kernel with four landmarks
# per thread), world of one on RCCL: per-scan wall time after 4 warm-up scans.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_shard32k}; mkdir -p $out/d
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29631 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 python3 tests/rowshard_gpu_worker.py --out $out/d --N 32768 --T 4 --scans 16 --precision 1 --backend nccl --native > $out/run.log 2>&1 || exit 1
python3 -c "import numpy as np; d=np.load('$out/d/rank0.npz'); t=d['times'][4:]; print('N=32768 one-call scan median', round(float(np.median(t))*1e3, 4), 'ms min', round(float(t.min())*1e3, 4))" > $out/summary.txt
rm -f $out/d/rank0.npz
cat $out/summary.txt
