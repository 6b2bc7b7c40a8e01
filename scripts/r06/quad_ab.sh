# Timing variants of the quad flush (xp_q*.so, built by -D switches): bench lines at N = 4096, T = 20
# usage: TAG=<tag> VARIANTS="qL4 qD4 ..." bash scripts/r06/quad_ab.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_quadab}; mkdir -p $out
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $out/q_$r.json 2> $out/q_$r.err || exit 1
  for v in $VARIANTS; do
    SLAM_EKF_LIB=slam_ros_amd/lib/xp_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $out/${v}_$r.json 2> $out/${v}_$r.err || exit 1
  done
done
