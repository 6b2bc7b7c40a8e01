# One bench configuration end to end on the GPU box: kernel trace stats and the PMC passes (each its
# own run), the counter summary (traffic.json for this library build, written next to the runs),
# then the bench line with its parity and CPU-baseline legs reading that traffic file.
# usage: TAG=<tag> bash scripts/r05/config_line.sh <bench args...>   → gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-line}
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT/profile
echo "start $(date +%s)" > $OUT/status
timeout -k 10 240 python bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/kt.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/fetch -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/write -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/write.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/sq -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/sq.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_FMA_F64 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/insts -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/insts.log 2>&1 && \
timeout -k 10 120 python scripts/pmc_summary.py $TAG $OUT/profile > $OUT/summary.log 2>&1 && \
timeout -k 10 400 python bench.py --traffic-json $OUT/profile/traffic.json "$@" > $OUT/bench_full.json 2> $OUT/bench_full.err
rc=$?
echo "exit $rc" >> $OUT/status
exit $rc
