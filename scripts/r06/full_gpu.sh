# The whole GPU suite, then the drop-in timing. usage: TAG=<tag> bash scripts/r06/full_gpu.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_full}; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || exit 1
TAG=${TAG:-r06_full}_dropin bash scripts/r06/dropin.sh
