# Phase timers of the association kernel in the drop-in's configuration (N = 100, E = 1, fp64, T = 1)
set -o pipefail
out=gpurun_out/${TAG:-r06_dprobe}; mkdir -p $out
PROBE_E=1 PROBE_PREC=f64 PROBE_ARITH=exact timeout -k 10 200 python scripts/assoc_probe.py 100:1 100:4 > $out/probe.json 2> $out/probe.err || exit 1
