# Counter profiles (kernel trace, FETCH/WRITE, SQ) of the bench configurations, one tag each:
# PROF_SET="n4096 n1024 n256 f16 f64" (default all), PREFIX=r03 → gpurun_out/<PREFIX>_<name>
set -o pipefail
cd $GRAFT_REPO_ROOT
PREFIX=${PREFIX:-r03}
for c in ${PROF_SET:-n4096 n1024 n256 f16 f64}; do
  case $c in
    n4096) args="--steps 20 --warmup 5";;
    n1024) args="--capacity 1024 --steps 40 --warmup 20";;
    n256)  args="--capacity 256 --steps 40 --warmup 20";;
    f16)   args="--precision f16 --steps 20 --warmup 5";;
    f16e)  args="--precision f16 --arith exact --steps 20 --warmup 5";;
    f64)   args="--precision f64 --steps 20 --warmup 5";;
  esac
  TAG=${PREFIX}_$c bash scripts/pmc_profile.sh $args || exit 1
done
