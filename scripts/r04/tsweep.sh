# split-fp16 flush interval sweep at the driver's 20 steps and at 48, then the f16x3 bench-config
# parity tests. usage: bash scripts/r04/tsweep.sh → gpurun_out/r04_tsweep*/
set -o pipefail
cd $GRAFT_REPO_ROOT
C="--arith f16x3 --flush-interval 16;--arith f16x3 --flush-interval 20;--arith f16x3 --flush-interval 24"
STEPS=20 TAG=r04_tsweep20 CONFIGS="$C" bash scripts/r04/ab.sh && \
STEPS=48 TAG=r04_tsweep48 CONFIGS="$C" bash scripts/r04/ab.sh && \
timeout -k 10 500 python -u -m pytest tests/test_bench_config.py -m gpu -v -k f16x3 --timeout 240 --timeout-method thread > gpurun_out/r04_tsweep48/pytest.log 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json gpurun_out/r04_tsweep48/ 2>/dev/null
exit $rc
