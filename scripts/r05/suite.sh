#!/bin/bash
# the whole GPU suite, smoke, and the flush-interval sweep at N = 256 / 1024
set -o pipefail
out=gpurun_out/${TAG:-r05_suite}; mkdir -p $out
rm -f gpurun_out/bench_config_parity.json
timeout -k 10 1000 python -u -m pytest tests -m gpu ${XFLAG--x} -v --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
cp gpurun_out/bench_config_parity.json $out/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit 1
if [ "${SWEEP:-1}" = "1" ]; then bash scripts/r05/tsweep.sh; fi
