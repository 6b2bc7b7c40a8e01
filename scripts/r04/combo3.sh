# fp16-storage and fp64 profiled lines, then the association phase timers in both worlds (f16x3).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04_probe
LINES="r04_f16|--steps 20 --warmup 5 --precision f16;r04_f64|--steps 20 --warmup 5 --precision f64" bash scripts/r04/lines.sh && \
PROBE_ARITH=f16x3 timeout -k 10 150 python scripts/assoc_probe.py 4096:20 1024:20 > gpurun_out/r04_probe/bench_world.txt 2>&1 && \
PROBE_ARITH=f16x3 PROBE_WORLD=survey timeout -k 10 150 python scripts/assoc_probe.py 4096:20 > gpurun_out/r04_probe/survey_world.txt 2>&1 && \
TAG=r04_survey3 bash scripts/r04/survey.sh
