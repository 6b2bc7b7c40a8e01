# iteration (tests, stamps, bench) then counter profiles of $PROF_SET (scripts/r03/profiles.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r03_iter}
bash scripts/r03/iter.sh || exit 1
PREFIX=${PREFIX:-$TAG} bash scripts/r03/profiles.sh
