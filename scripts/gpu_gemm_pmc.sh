#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, kernel-trace only) on one GEMM shape, ours vs hipBLASLt.
OUT=gpurun_out/${1:-gemm_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
SHAPE="${2:-1 16384 2048 8192}"

PMC="${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE}"
for who in ours blas; do
  timeout -s KILL 90 rocprofv3 --pmc $PMC --kernel-trace -d $OUT/$who -o p1 --output-format csv -- python3 scripts/gemm_one.py $who $SHAPE 5 > $OUT/$who.p1.log 2>&1 || { echo "pmc $who failed"; tail -5 $OUT/$who.p1.log; exit 1; }
done
echo ok
