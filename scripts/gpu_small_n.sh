# BASELINE configs 2 and 3 (N=256, N=1024 at one GPU): bench lines, then rocprof stats and the
# FETCH/WRITE passes at N=1024; every GPU step time-limited, stop at the first failure
set -o pipefail
mkdir -p gpurun_out/small
export TMPDIR=/tmp
for n in 256 1024; do
  timeout -k 10 200 python bench.py --capacity $n > gpurun_out/small/bench_n$n.json 2> gpurun_out/small/bench_n$n.err || { tail -20 gpurun_out/small/bench_n$n.err; exit 1; }
done
B="python3 bench.py --no-cpu --capacity 1024"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/small/kt -o run --output-format csv -- $B > gpurun_out/small/kt.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/small/fetch -o run --output-format csv -- $B > gpurun_out/small/fetch.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/small/write -o run --output-format csv -- $B > gpurun_out/small/write.log 2>&1 && \
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/small/sq -o run --output-format csv -- $B > gpurun_out/small/sq.log 2>&1
rc=$?; echo "exit $rc"; exit $rc
