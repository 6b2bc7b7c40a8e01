# Several profiled bench lines in one call (scripts/r05/config_line.sh each; a failure ends the call).
# usage: LINES="tag1|args1;tag2|args2" bash scripts/r05/lines.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
IFS=';' read -ra LS <<< "$LINES"
for item in "${LS[@]}"; do
  tag="${item%%|*}"; args="${item#*|}"
  TAG=$tag bash scripts/r05/config_line.sh $args || { echo "line $tag failed"; exit 1; }
done
echo "lines done"
