# CPU baselines (B0 faithful 1 core incl. N = 4096 once, B1 OpenMP and 1 core) on the GPU box's
# host, with a heartbeat file so the long single B0 update at N = 4096 is not taken for a hang
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 50; date >> gpurun_out/cpu_heartbeat; done ) &
hb=$!
timeout -k 10 1000 python -u scripts/cpu_baselines.py all > gpurun_out/r02_cpu_baselines.jsonl 2> gpurun_out/cpu_baselines.err
rc=$?
kill $hb
exit $rc
