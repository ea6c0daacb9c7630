#!/bin/bash
# Wave-state + clock counters on fc1 dgrad (dy·Wᵀ 16384x2048x8192): W8, W4 and hipBLASLt.
OUT=gpurun_out/${1:-r4b}
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="1 16384 2048 8192"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
for who in w8 w4 blas; do
  case $who in w8) W=0; B=ours;; w4) W=2; B=ours;; blas) W=0; B=blas;; esac
  for p in 1 2 3; do
    eval PMC=\$P$p
    PRA_GEMM_W4=$W timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace -d $OUT/$who -o p$p --output-format csv -- python3 scripts/gemm_one.py $B $SHAPE 6 > $OUT/$who.p$p.log 2>&1 || { echo "pmc $who p$p failed"; tail -5 $OUT/$who.p$p.log; exit 1; }
  done
done
echo ok
