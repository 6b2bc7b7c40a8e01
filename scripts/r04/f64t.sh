# fp64 bench line at T = 4, 6, 8 on the MFMA-replay build (the on-read replay no longer grows
# 35 µs per pending step), driver's 20 steps, each twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
C="--precision f64 --flush-interval 4;--precision f64 --flush-interval 6;--precision f64 --flush-interval 8"
STEPS=20 TAG=r04_f64t CONFIGS="$C" bash scripts/r04/ab.sh
