# Flush arithmetic / T / wave-count A/B (scripts/r04/ab.sh) and the association phase timers for
# both split arithmetics. usage: bash scripts/r04/measure1.sh → gpurun_out/r04_m1/
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-r04_m1}
mkdir -p $OUT
TAG=${TAG:-r04_m1} VARIANTS="${VARIANTS:-base xp_f16w2}" CONFIGS="${CONFIGS:---arith f16x3;--arith f16x3 --flush-interval 16;--arith bf16x6}" bash scripts/r04/ab.sh && \
timeout -k 10 150 python scripts/assoc_probe.py 4096:12 1024:12 > $OUT/probe_bf.txt 2>&1 && \
PROBE_ARITH=f16x3 timeout -k 10 150 python scripts/assoc_probe.py 4096:12 1024:12 > $OUT/probe_f16.txt 2>&1
rc=$?
echo "measure1 exit $rc" >> $OUT/status
exit $rc
