#!/bin/bash
# Op tables by Python call site for the GPT and BERT steps (where the fill / copy / reduce
# kernels come from), plus a rocprofv3 kernel table of the BERT step.
OUT=gpurun_out/${1:-r4l}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4; if fatal $rc; then exit $rc; fi; }
step gpt 300 python bench.py --steps 6 --warmup 3 --profile-dir $OUT/gpt_ops
step bert 300 python bench.py --model bert-base --steps 10 --warmup 3 --profile-dir $OUT/bert_ops
exit 0
