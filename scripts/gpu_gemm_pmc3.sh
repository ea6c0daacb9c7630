#!/bin/bash
# Wave-state counters on the fc1 dgrad shape (dy·Wᵀ, 16384x2048x8192): W8, W4 and hipBLASLt.
# Pass 1 splits wave time into waiting / issue-stalled / active; pass 2 the memory side.
OUT=gpurun_out/${1:-gemm_pmc3}
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="1 16384 2048 8192"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for who in w8 w4 blas; do
  case $who in w8) W=0; B=ours;; w4) W=2; B=ours;; blas) W=0; B=blas;; esac
  for p in 1 2; do
    eval PMC=\$P$p
    PRA_GEMM_W4=$W timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace -d $OUT/$who -o p$p --output-format csv -- python3 scripts/gemm_one.py $B $SHAPE 5 > $OUT/$who.p$p.log 2>&1 || { echo "pmc $who p$p failed"; tail -5 $OUT/$who.p$p.log; exit 1; }
  done
done
echo ok
