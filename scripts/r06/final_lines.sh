# Round 6's final profiled lines (scripts/r05/config_line.sh each), one call
set -o pipefail
cd $GRAFT_REPO_ROOT
LINES="r06_final_n4096|--steps 20 --warmup 5;r06_final_n1024|--steps 20 --warmup 5 --capacity 1024;r06_final_n256|--steps 20 --warmup 5 --capacity 256;r06_final_f16|--steps 20 --warmup 5 --precision f16;r06_final_f64|--steps 20 --warmup 5 --precision f64;r06_final_survey|--steps 20 --warmup 5 --world survey" bash scripts/r05/lines.sh
