# PMC passes on the sequential bench (the flush kernel runs alone on the chip)
set -o pipefail
mkdir -p gpurun_out/ctr
export TMPDIR=/tmp
rm -rf gpurun_out/ctr/*
T=${T:-4}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ctr/sq -o run --output-format csv -- python3 bench.py --no-cpu --pipeline 0 --flush-interval $T --steps 16 --warmup 4 > gpurun_out/ctr_sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_F32 SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/ctr/ins -o run --output-format csv -- python3 bench.py --no-cpu --pipeline 0 --flush-interval $T --steps 16 --warmup 4 > gpurun_out/ctr_ins.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
