# A/B bench lines of library variants × bench arguments on one box, each combination twice in
# alternating order. VARIANTS="base xp_name ..." (base = libslam_ekf.so), CONFIGS="args1;args2;..."
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r04_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
IFS=';' read -ra CFGS <<< "${CONFIGS:---arith f16x3}"
for rep in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/$v.so; fi
    for i in "${!CFGS[@]}"; do
      SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps ${STEPS:-48} --warmup 50 --no-cpu ${CFGS[$i]} > $OUT/bench_${v}_c${i}_$rep.json 2> $OUT/bench_${v}_c${i}_$rep.err || { echo "fail $v $i" > $OUT/status; exit 1; }
    done
  done
done
echo done > $OUT/status
