# instances per GPU at N = 256 / 1024 / 4096: association kernels fill more CUs (one workgroup per
# CU, G = ceil(N / 192) per instance); headline stays E = 8 (BASELINE config 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-occ}
mkdir -p $OUT
for cfg in "1024 8" "1024 16" "1024 40" "256 8" "256 64" "256 128" "4096 11" "4096 8"; do
  set -- $cfg
  timeout -k 10 150 python bench.py --steps 200 --warmup 20 --no-cpu --capacity $1 --instances $2 > $OUT/n$1_e$2.json 2> $OUT/n$1_e$2.err || exit 1
done
for f in $OUT/*.json; do python scripts/show_bench.py $f; done > $OUT/summary.txt 2>&1
