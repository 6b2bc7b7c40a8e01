set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f64ab
for v in 0 9 0 9; do
  EKF_FLUSH_VARIANT=$v timeout -k 10 120 python bench.py --no-cpu --precision f64 --flush-interval 4 --steps 40 --warmup 5 > gpurun_out/f64ab/b_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/f64ab/b_$v.json')); print('variant $v', d['value'], d['kernel_ms']['flush'])" >> gpurun_out/f64ab/summary.txt
done
EKF_FLUSH_VARIANT=9 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "f64_wave" > gpurun_out/f64ab/pytest9.log 2>&1
echo "pytest9 rc=$?" >> gpurun_out/f64ab/summary.txt
