# The split-fp16 quad flush (EKF_OPT_FLUSH_FORM = 44): bit-identity tests against the 2 x 2 form,
# then bench lines of both forms alternating, then a kernel-trace profile of the quad form.
# usage: TAG=<tag> bash scripts/r06/quad.sh
set -o pipefail
out=gpurun_out/${TAG:-r06_quad}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "quad_flush" > $out/pytest.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $out/q_$r.json 2> $out/q_$r.err || exit 1
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu > $out/w_$r.json 2> $out/w_$r.err || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu --flush-form 44 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1
