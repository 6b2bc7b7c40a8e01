# Bench lines of record for DESIGN §5 (one box): fp16 / fp64 / N=1024 / N=256, the association's
# bad cases (speculate option 0 and 2) and SURVEY §8d's world, then tests/diag/assoc_cases.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_measure}
O=gpurun_out/$TAG
mkdir -p $O
run() { name=$1; shift; timeout -k 10 180 python bench.py --no-cpu --steps 48 --warmup 20 "$@" > $O/$name.json 2> $O/$name.err || { echo "fail $name" >> $O/status; exit 1; }; }
run f32
run f16 --precision f16
run f16_t8 --precision f16 --flush-interval 8
run f64 --precision f64
run n1024 --capacity 1024
run n256 --capacity 256
run spec0 --speculate 0
run spec2 --speculate 2
run survey --world survey
timeout -k 10 600 python tests/diag/assoc_cases.py --k 24 --w 12 > $O/assoc_cases.txt 2>&1 || { echo "fail assoc_cases" >> $O/status; exit 1; }
echo done >> $O/status
