# Copy a config_line.sh result (gpurun_out/<tag>/) into profiles/<dest>/ with its paths rewritten:
# the profiled bench line (bench.json), counter summaries, traffic.json, kernel stats and the raw
# counter CSVs. usage: bash scripts/r04/keep_line.sh <tag> [dest]
set -e
TAG=$1; DEST=${2:-$1}
SRC=gpurun_out/$TAG
OUT=profiles/$DEST
mkdir -p $OUT
cp $SRC/profile/counters_avg_per_dispatch.json $SRC/profile/kernel_stats.csv $OUT/
[ -f $SRC/profile/scan_instructions.json ] && cp $SRC/profile/scan_instructions.json $OUT/
cp $SRC/summary.log $OUT/
for p in fetch write sq insts; do cp $SRC/$p/run_counter_collection.csv $OUT/${p}_counter_collection.csv; done
sed "s#gpurun_out/$TAG/profile/#profiles/$DEST/#g; s#profiles/$TAG/#profiles/$DEST/#g" $SRC/profile/traffic.json > $OUT/traffic.json
sed "s#gpurun_out/$TAG/profile/#profiles/$DEST/#g; s#profiles/$TAG/#profiles/$DEST/#g" $SRC/bench_full.json > $OUT/bench.json
echo "kept $SRC -> $OUT"
