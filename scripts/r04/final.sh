# Round-end evidence on one build: the GPU suite, smoke and the driver's bench command (check.sh;
# PART=check), then every configuration's profiled line (config_line.sh via lines.sh; PART=lines).
# Without PART both, in one call.
set -o pipefail
cd $GRAFT_REPO_ROOT
if [ "${PART:-all}" != lines ]; then
  PYTEST_S=700 TAG=r04_final_check bash scripts/r04/check.sh; r1=$?
  if [ $r1 -ne 0 ] && [ $r1 -ne 1 ]; then exit $r1; fi
  cp gpurun_out/bench_config_parity.json gpurun_out/r04_final_check/ 2>/dev/null
fi
if [ "${PART:-all}" != check ]; then
  LINES="r04_final_n4096|--steps 20 --warmup 5;r04_final_n1024|--steps 20 --warmup 5 --capacity 1024;r04_final_n256|--steps 20 --warmup 5 --capacity 256;r04_final_f16|--steps 20 --warmup 5 --precision f16;r04_final_f64|--steps 20 --warmup 5 --precision f64;r04_final_survey|--steps 20 --warmup 5 --world survey" bash scripts/r04/lines.sh
fi
