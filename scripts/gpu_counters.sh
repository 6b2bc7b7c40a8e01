# PMC passes on the sequential T=4 bench (flush kernel runs alone on the chip)
set -o pipefail
mkdir -p gpurun_out/ctr
export TMPDIR=/tmp
rm -rf gpurun_out/ctr/*
V=${EKF_FLUSH_VARIANT:-0}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ctr/sq -o run --output-format csv -- python3 bench.py --no-cpu --pipeline 0 --flush-interval 4 --steps 16 --warmup 4 > gpurun_out/ctr_sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ctr/tcc -o run --output-format csv -- python3 bench.py --no-cpu --pipeline 0 --flush-interval 4 --steps 16 --warmup 4 > gpurun_out/ctr_tcc.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ctr/lds -o run --output-format csv -- python3 bench.py --no-cpu --pipeline 0 --flush-interval 4 --steps 16 --warmup 4 > gpurun_out/ctr_lds.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
