# association phase stamps + driver-command bench on the current build, then the bench on each
# $VARIANTS library (timing experiments)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_base}
mkdir -p gpurun_out/$TAG
timeout -k 10 240 python scripts/assoc_probe.py ${PROBE_CFGS:-4096:12 4096:8 1024:8} > gpurun_out/$TAG/probe.txt 2>&1 && \
timeout -k 10 180 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
for v in $VARIANTS; do
  SLAM_EKF_LIB=slam_ros_amd/lib/$v.so timeout -k 10 120 python bench.py --steps 48 --warmup 200 --no-cpu > gpurun_out/$TAG/bench_$v.json 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --steps 48 --warmup 200 --no-cpu > gpurun_out/$TAG/bench_default48.json 2>&1
rc=$?
echo "exit $rc" > gpurun_out/$TAG/status
exit $rc
