#!/bin/bash
# TS-schedule GEMM configurations vs the defaults and hipBLASLt on the GPT shapes.
OUT=gpurun_out/${1:-r4c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/gemm_lds_bench.py --w4 --ts > $OUT/gemm_ts.log 2>&1; rc=$?
echo "[gemm rc=$rc]"; tail -n 22 $OUT/gemm_ts.log
exit $rc
