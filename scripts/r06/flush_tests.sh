# Flush-form tests after a kernel change: every flush parity / bit-identity test, then bench lines
# of the default and the quad form. usage: TAG=<tag> bash scripts/r06/flush_tests.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_flush}; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "flush or quad or wave or bf16 or f16" > $out/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > $out/bench.json 2> $out/bench.err || exit 1
timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $out/quad.json 2> $out/quad.err || exit 1
