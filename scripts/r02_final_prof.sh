# Final PMC profiles of the three bench lines (f32 default, fp64 T = 4, fp16 T = 8): bench line,
# kernel trace stats, FETCH / WRITE / SQ passes each in its own run (scripts/pmc_profile.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r02_final bash scripts/pmc_profile.sh --steps 20 --warmup 5 && \
TAG=r02_final_f64 bash scripts/pmc_profile.sh --precision f64 --flush-interval 4 --steps 40 --warmup 5 && \
TAG=r02_final_f16 bash scripts/pmc_profile.sh --precision f16 --steps 20 --warmup 5
