# The speculative guesses in fp64 (EKF_GUESS_T=double, xp_g64.so) against fp32 (the product):
# the SURVEY world's restart distribution (scripts/r06/restart_diag.py) and bench lines (survey,
# default N = 4096), two repetitions.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_guess}; mkdir -p $out
SLAM_EKF_LIB=slam_ros_amd/lib/xp_g64.so timeout -k 10 300 python3 scripts/r06/restart_diag.py 20 200 60 > $out/diag20_g64.json 2> $out/diag20_g64.err || exit 1
for rep in 1 2; do
  for lib in product g64; do
    if [ $lib = product ]; then L=slam_ros_amd/lib/libslam_ekf.so; else L=slam_ros_amd/lib/xp_$lib.so; fi
    for cfg in "survey|--world survey" "n4096|"; do
      name="${cfg%%|*}"; args="${cfg#*|}"
      SLAM_EKF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu $args > $out/${lib}_${name}_$rep.json 2> $out/${lib}_${name}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$out/${lib}_${name}_$rep.json').read().strip().splitlines()[-1]); print('$lib $name rep $rep', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4), 'scan', round(d['kernel_ms']['scan']*1e3,1))" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
