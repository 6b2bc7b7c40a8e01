# fp64 MFMA replay of pending steps: its identity tests and the fp64 / deferred / rollback parity
# tests, then the fp64 bench line (twice) and its association probe.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04_combo6
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_rollback.py tests/test_bench_config.py -m gpu -v -k "f64 or deferred or rollback or singular or speculative or prec0 or 0-" --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest $rc" > $OUT/status
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --precision f64 > $OUT/bench_f64_$i.json 2> $OUT/bench_f64_$i.err || exit 5
done
PROBE_PREC=f64 timeout -k 10 150 python scripts/assoc_probe.py 4096:4 > $OUT/probe_f64.txt 2>&1 || exit 6
echo "done" >> $OUT/status
