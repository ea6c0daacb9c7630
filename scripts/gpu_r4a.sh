#!/bin/bash
# Round-4 entry: GEMM configuration table (all in-tree configs vs hipBLASLt) on the GPT shapes.
OUT=gpurun_out/${1:-r4a}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_lds_bench.py --w4 > $OUT/gemm_w4.log 2>&1; rc=$?
echo "[gemm rc=$rc]"; tail -n 25 $OUT/gemm_w4.log
exit $rc
