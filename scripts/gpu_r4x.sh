#!/bin/bash
# fc2 dgrad + dGELU + bias-grad epilogue (in-tree TS / persistent) vs hipBLASLt + bias_gelu_bwd_db.
OUT=gpurun_out/${1:-r4x}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3; if fatal $rc; then exit $rc; fi; }
step ts 200 python scripts/gemm_lds_bench.py --fused
step pts 200 python scripts/gemm_lds_bench.py --fused --pts
exit 0
