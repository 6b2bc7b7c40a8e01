# fp64 association changes: the fp64 bit-identity / parity tests, then the phase timers and bench line
# usage: TAG=<tag> bash scripts/r06/f64_tests.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_f64t}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "f64 or speculative_association_identical or trajectory or singular" > $out/pytest.log 2>&1 || exit 1
PROBE_PREC=f64 PROBE_ARITH=exact timeout -k 10 200 python scripts/assoc_probe.py 4096:8 > $out/probe.json 2> $out/probe.err || exit 1
for r in 1 2; do
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu --precision f64 > $out/bench_$r.json 2> $out/bench_$r.err || exit 1
done
