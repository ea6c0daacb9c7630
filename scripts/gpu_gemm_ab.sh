#!/bin/bash
# In-tree GEMM vs hipBLASLt on every GPT-1.3B GEMM shape (+ fused epilogue vs separate), one process.
OUT=gpurun_out/${1:-gemm_ab}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 env PRA_GEMM=mfma python scripts/gemm_lds_bench.py > $OUT/gemm.log 2>&1; rc=$?
tail -30 $OUT/gemm.log
[ $rc = 0 ] && { timeout -k 10 200 env PRA_GEMM=mfma python scripts/gemm_lds_bench.py --fused > $OUT/fused.log 2>&1; rc=$?; tail -8 $OUT/fused.log; }
exit $rc
