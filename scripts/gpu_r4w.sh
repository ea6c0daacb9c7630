#!/bin/bash
# End-of-round GPT-1.3B per-step kernel table (rocprofv3 kernel trace, timed steps only) + bench.
OUT=gpurun_out/${1:-r4w}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
step gpt 300 python bench.py --steps 20 --warmup 5
step gpt_prof 400 rocprofv3 --kernel-trace -d $OUT/gpt_prof -o gpt -- python bench.py --steps 10 --warmup 3
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
