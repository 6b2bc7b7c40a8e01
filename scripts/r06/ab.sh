# A/B of the association kernel: targeted bit-identity / parity tests on the new build, then bench
# lines of the previous build (xp_base.so) and this tree's, alternating, and the phase timers
# (xp_stamps128.so). usage: TAG=<tag> bash scripts/r06/ab.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_ab}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "speculative_association_identical or narrow_scan or hot_scan or gate_storage or active_flush" \
  tests/test_bench_config.py -k "f16x3 or survey_world_association or t8 or speculative or narrow" \
  tests/test_rollback.py tests/test_rowshard_gpu.py > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
  SLAM_EKF_LIB=slam_ros_amd/lib/xp_base.so timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $out/base_$r.json 2> $out/base_$r.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $out/new_$r.json 2> $out/new_$r.err || exit 1
done
SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps128.so PROBE_ARITH=f16x3 timeout -k 10 200 python scripts/assoc_probe.py 4096:20 > $out/probe4096.json 2> $out/probe4096.err
