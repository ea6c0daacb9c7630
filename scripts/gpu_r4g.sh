#!/bin/bash
# TS (hipBLASLt-shaped) K-loop vs default W4/W8 on the 15 GPT shapes; stamps; GPT bench.
OUT=gpurun_out/${1:-r4g}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 25; if fatal $rc; then exit $rc; fi; }
step mha2 200 python -u scripts/debug_mha2.py
step ts 300 python -u scripts/gemm_lds_bench.py --w4 --ts
step stamps 200 python -u scripts/gemm_stamps.py
exit 0
