# Default bench (with CPU baseline), then kernel-trace stats and the two PMC passes of the same
# command; every GPU step under its own time limit, chained so that a failure stops the script.
set -o pipefail
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
rm -rf gpurun_out/prof/*
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof/kt -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof/fetch -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof/write -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/prof/sq -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_sq.log 2>&1
rc=$?
echo "exit $rc" > gpurun_out/profile.status
exit $rc
