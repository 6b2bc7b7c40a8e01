# Full GPU parity suite on the default build, repeated fp32/fp16 bench lines (flush forms A/B),
# SQ counters of the fp32 and fp16 flush. Every GPU step time-limited; the first failure ends it.
set -o pipefail
mkdir -p gpurun_out/sqab
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for rep in 1 2; do CFGS="0:0:8 0:83:8 0:0:8:f16" bash scripts/gpu_sweep.sh || exit 1; done
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
for prec in f32 f16; do
  timeout -k 10 120 rocprofv3 --pmc $SQ --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/sqab/$prec -o run --output-format csv -- python3 bench.py --no-cpu --precision $prec --steps 64 --warmup 64 > gpurun_out/sqab/$prec.log 2>&1 || { echo "pmc $prec failed"; tail -20 gpurun_out/sqab/$prec.log; exit 1; }
done
python scripts/wprof_summary.py gpurun_out/sqab
