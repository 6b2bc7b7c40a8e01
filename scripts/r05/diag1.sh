#!/bin/bash
# MFMA accumulation rounding probe; split flush decomposition (XP builds); survey parity with the
# exact per-element replay under the split arithmetics
set -o pipefail
out=gpurun_out/r05_d1; mkdir -p $out
timeout -k 10 60 ./scripts/probe/mfma_acc_error > $out/probe.txt 2>&1 &&
for v in base xp_notiles xp_noops; do
  if [ $v = base ]; then lib=slam_ros_amd/lib/libslam_ekf.so; else lib=slam_ros_amd/lib/$v.so; fi
  SLAM_EKF_LIB=$lib timeout -k 10 150 python bench.py --steps 40 --warmup 20 --no-cpu > $out/bench_$v.json 2> $out/bench_$v.err || exit 1
done &&
XP_ARITH=f16x3 XP_T=20 SLAM_EKF_LIB=slam_ros_amd/lib/xp_stamps.so timeout -k 10 120 python scripts/xp_flush_stamps.py > $out/stamps.json 2> $out/stamps.err &&
timeout -k 10 500 python -u tests/diag/survey_parity.py f16x3:16:mfma_replay=0,bf16x6:16:mfma_replay=0 0 48 > $out/sp_norep.jsonl 2> $out/sp_norep.err
