# Compiler scheduling strategies for the whole library (xp_trk: AMDGPU register-pressure trackers,
# xp_milp: max-ilp, xp_iilp: iterative-ilp) against the product: bench lines at N = 4096 and
# N = 1024 (scan and flush HIP-event times in each line), two repetitions.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_sched}; mkdir -p $out
for rep in 1 2; do
  for lib in product trk milp iilp; do
    if [ $lib = product ]; then L=slam_ros_amd/lib/libslam_ekf.so; else L=slam_ros_amd/lib/xp_$lib.so; fi
    for cfg in "n4096|" "n1024|--capacity 1024"; do
      name="${cfg%%|*}"; args="${cfg#*|}"
      SLAM_EKF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu $args > $out/${lib}_${name}_$rep.json 2> $out/${lib}_${name}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$out/${lib}_${name}_$rep.json').read().strip().splitlines()[-1]); print('$lib $name rep $rep', round(d['value'],1), 'ms/step', round(d['ms_per_step'],4), 'scan', round(d['kernel_ms']['scan']*1e3,2), 'flush', round(d['kernel_ms']['flush'],4))" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
