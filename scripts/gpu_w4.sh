#!/bin/bash
# W4 (4-wave, 128x128 per wave) GEMM configuration vs W8 vs hipBLASLt, + fused epilogues.
OUT=gpurun_out/${1:-w4}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 25 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step w4 300 python scripts/gemm_lds_bench.py --w4
step fused8 120 python scripts/gemm_lds_bench.py --fused
step fused4 120 python scripts/gemm_lds_bench.py --fused --w4
exit 0
