#!/bin/bash
# GEMM phase stamps (diagnostic build) on the GPT shapes.
OUT=gpurun_out/${1:-r4d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/gemm_stamps.py > $OUT/stamps.log 2>&1; rc=$?
echo "[stamps rc=$rc]"; cat $OUT/stamps.log | grep -v amdgpu.ids
exit $rc
