# association phase stamps only: the bench's arithmetic, then the exact one
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_probe}
mkdir -p gpurun_out/$TAG
timeout -k 10 240 python scripts/assoc_probe.py ${PROBE_CFGS:-4096:12 1024:8} > gpurun_out/$TAG/probe.txt 2>&1 && \
PROBE_ARITH=exact timeout -k 10 240 python scripts/assoc_probe.py 4096:12 >> gpurun_out/$TAG/probe.txt 2>&1
