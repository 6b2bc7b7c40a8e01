# a failed verdict keeps the lines before the first violating one. The association
# GPU tests (bit identity against the sequential path, rollback, the survey world against the
# oracle), then bench lines of this build against the previous commit's (xp_head.so): the survey
# world and the default N = 4096 line, two repetitions each.
set -o pipefail
cd $GRAFT_REPO_ROOT
out=gpurun_out/${TAG:-r06_restart}; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py tests/test_bench_config.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
cp gpurun_out/bench_config_parity.json $out/ 2>/dev/null
for rep in 1 2; do
  for lib in product head; do
    if [ $lib = product ]; then L=slam_ros_amd/lib/libslam_ekf.so; else L=slam_ros_amd/lib/xp_$lib.so; fi
    for cfg in "survey|--world survey" "n4096|"; do
      name="${cfg%%|*}"; args="${cfg#*|}"
      SLAM_EKF_LIB=$L timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu $args > $out/${lib}_${name}_$rep.json 2> $out/${lib}_${name}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$out/${lib}_${name}_$rep.json').read().strip().splitlines()[-1]); print('$lib $name rep $rep', round(d['value'],1), d['unit'], 'ms/step', round(d['ms_per_step'],4))" >> $out/summary.txt
    done
  done
done
cat $out/summary.txt
