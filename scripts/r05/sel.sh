#!/bin/bash
# a selection of GPU tests: SEL = pytest -k expression, FILES = test files
set -o pipefail
out=gpurun_out/${TAG:-r05_sel}; mkdir -p $out
timeout -k 10 ${TLIM:-900} python -u -m pytest ${FILES:-tests} -m gpu -k "${SEL}" -v --timeout 400 --timeout-method thread > $out/pytest.log 2>&1
