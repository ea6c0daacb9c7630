#!/bin/bash
# BERT static step op table (no HIP graph, so the profiler sees each op) + rocprofv3 kernel
# table of the graph-replayed step.
OUT=gpurun_out/${1:-r4m}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3; if fatal $rc; then exit $rc; fi; }
step bert_nog 300 python bench.py --model bert-base --steps 5 --warmup 3 --no-graph --profile-dir $OUT/bert_ops
step bert_prof 300 rocprofv3 --kernel-trace --stats -d $OUT/bert_prof -o bert -- python bench.py --model bert-base --steps 30 --warmup 3
exit 0
