#!/bin/bash
# Two counter passes on the fc1 dgrad shape (dy·Wᵀ, 16384x2048x8192), ours vs hipBLASLt.
OUT=gpurun_out/${1:-gemm_pmc2}
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="1 16384 2048 8192"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM"
for who in ours blas; do
  for p in 1 2; do
    eval PMC=\$P$p
    timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace -d $OUT/$who -o p$p --output-format csv -- python3 scripts/gemm_one.py $who $SHAPE 5 > $OUT/$who.p$p.log 2>&1 || { echo "pmc $who p$p failed"; tail -5 $OUT/$who.p$p.log; exit 1; }
  done
done
echo ok
