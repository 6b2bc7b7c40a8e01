# phase probe of a variant library (results may be invalid: no assertions) vs the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-probe}
mkdir -p $OUT
timeout -k 10 120 python scripts/assoc_probe.py 4096:8 > $OUT/probe_a.txt 2>&1 && \
PROBE_NOASSERT=1 SLAM_EKF_LIB=$LIB timeout -k 10 120 python scripts/assoc_probe.py 4096:8 > $OUT/probe_b.txt 2>&1
