#!/bin/bash
# New GEMM: correctness + timing vs hipBLASLt; then a rocprofv3 kernel-stats pass.
OUT=gpurun_out/${1:-gemm_lds}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python scripts/gemm_lds_bench.py ${2:-} > $OUT/bench.log 2>&1; rc=$?
cat $OUT/bench.log | tail -25
exit $rc
