#!/bin/bash
# PMC passes (one counter group per run) over single GEMM launches (tests/diagnostics/gemm_one.py):
# stall / LDS / MFMA counters of a tile on a shape.  CONFIGS="M,N,K,tile[,epi] ..."; tile -2 = torch.mm (the
# hipBLASLt yardstick) on the same operands.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/gpmc
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_WAVES"
P3="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU"
for c in ${CONFIGS:-8192,8192,8192,20}; do
  IFS=, read -r M N K T E <<< "$c"
  tag=${c//,/_}
  for p in 1 2 3; do
    ctr=P$p
    ( timeout -s KILL 90 rocprofv3 --pmc ${!ctr} --kernel-trace -f csv -d gpurun_out/gpmc/${tag}_p$p -o run -- \
      python3 tests/diagnostics/gemm_one.py $M $N $K $T 4 ${E:-0} > gpurun_out/gpmc/${tag}_p$p.log 2>&1 )
    rc=$?; echo "$c pass $p rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/gpmc/${tag}_p$p.log; exit $rc; }
  done
done
