# fp64 association phase timers and the fp64 bench line. usage: TAG=<tag> bash scripts/r06/f64_probe.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_f64}; mkdir -p $out
PROBE_PREC=f64 PROBE_ARITH=exact timeout -k 10 200 python scripts/assoc_probe.py 4096:8 > $out/probe.json 2> $out/probe.err || exit 1
timeout -k 10 150 python bench.py --steps 20 --warmup 5 --no-cpu --precision f64 > $out/bench.json 2> $out/bench.err || exit 1
