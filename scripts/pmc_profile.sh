# Profile one bench configuration: the bench line, the kernel-trace stats, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE and the SQ counters each in its own pass, MI355X_MICROARCH.md HBM
# section). usage: TAG=<tag> bash scripts/pmc_profile.sh <bench args...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-prof}
OUT=gpurun_out/$TAG
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 240 python bench.py --no-cpu "$@" > $OUT/bench.json 2> $OUT/bench.err && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/kt -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/kt.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/fetch -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/fetch.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/write -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/write.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/sq -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/sq.log 2>&1
rc=$?
# optional L2 pass (PMC_L2=1): hits and misses of the flush's operand and tile reads
if [ $rc -eq 0 ] && [ "${PMC_L2:-0}" = "1" ]; then
  timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/l2 -o run --output-format csv -- python3 bench.py --no-cpu "$@" > $OUT/l2.log 2>&1
  rc=$?
fi
echo "exit $rc" > $OUT/status
exit $rc
