#!/bin/bash
# ResNet-50 per-step kernel table (timed steps only).
OUT=gpurun_out/${1:-r4y}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
step rn_prof 400 rocprofv3 --kernel-trace -d $OUT/rn_prof -o rn -- python bench.py --model resnet50 --steps 10 --warmup 3
exit 0
