set -o pipefail
for b in 2 4 6 8 12; do
  for pipe in 0 1; do
    EKF_DD_BLOCKS_PER_CU=$b timeout -k 10 120 python bench.py --no-cpu --pipeline $pipe --steps 40 > gpurun_out/dd_${b}_${pipe}.json 2>/dev/null || exit 1
  done
done
