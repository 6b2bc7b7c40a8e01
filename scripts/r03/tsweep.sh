# flush interval sweep of the bench default (same library), each twice, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_tsweep}
mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for t in ${TS:-10 12 14 16}; do
    timeout -k 10 120 python bench.py --steps 48 --warmup 20 --no-cpu --flush-interval $t > gpurun_out/$TAG/bench_t${t}_$rep.json 2>&1 || exit 1
  done
done
