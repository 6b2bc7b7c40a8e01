# One box: the GPU suite + smoke + the driver's bench command (check.sh), then the SURVEY world.
set -o pipefail
cd $GRAFT_REPO_ROOT
PYTEST_S=700 TAG=${TAG:-r04_check2} bash scripts/r04/check.sh; r1=$?
if [ $r1 -ne 0 ] && [ $r1 -ne 1 ]; then exit $r1; fi
TAG=${STAG:-r04_survey2} bash scripts/r04/survey.sh
