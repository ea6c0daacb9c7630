#!/bin/bash
# Round 6 batch N: ResNet elementwise attribution; TunableOp dependency check; ResNet bench.
OUT=gpurun_out/${1:-r6n}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 25 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step resnet_ops 240 python scripts/r6_resnet_ops.py
step gpt_untuned 300 python bench.py --steps 20 --warmup 5 --no-tuned-gemms
step gpt_tuned 300 python bench.py --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
