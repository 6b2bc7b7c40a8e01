# counters of the wave flush (separate PMC passes, each time-limited): T=${T:-8}
set -o pipefail
mkdir -p gpurun_out/wprof
export TMPDIR=/tmp
B="python3 bench.py --no-cpu --flush-interval ${T:-8} --steps 48 --warmup 24"
EKF_FLUSH_VARIANT=8 timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/wprof/sq -o run --output-format csv -- $B > gpurun_out/wprof_sq.log 2>&1 && \
EKF_FLUSH_VARIANT=8 timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_F32 SQ_WAVES SQ_INST_CYCLES_VMEM --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/wprof/ins -o run --output-format csv -- $B > gpurun_out/wprof_ins.log 2>&1 && \
EKF_FLUSH_VARIANT=8 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/wprof/fetch -o run --output-format csv -- $B > gpurun_out/wprof_fetch.log 2>&1 && \
EKF_FLUSH_VARIANT=8 timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/wprof/tcc -o run --output-format csv -- $B > gpurun_out/wprof_tcc.log 2>&1
rc=$?; echo "exit $rc"; exit $rc
