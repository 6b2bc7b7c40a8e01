# the drop-in's per-call cost (scripts/r06/dropin_bench.py), then the kernel trace
# of the same C++ program under rocprofv3. → gpurun_out/${TAG:-r06_dropin}/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r06_dropin}; mkdir -p $out
timeout -k 10 300 python scripts/r06/dropin_bench.py $out 20 200 > $out/dropin.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/kt -o run --output-format csv -- $out/dropin_bench $out/scenario.txt $out/state.bin 20 200 > $out/kt.log 2>&1
