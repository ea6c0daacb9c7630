#!/bin/bash
# ERNIE-3.0 10B whole model on one GPU (the TP2 x PP4 path's single-GPU form) -- current numbers.
OUT=gpurun_out/${1:-r4ae}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-400; if fatal $rc; then exit $rc; fi; }
step ernie 900 python -u bench.py --model ernie-3.0-10b --steps 3 --warmup 1
exit 0
