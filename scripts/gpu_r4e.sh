#!/bin/bash
# Round-4 checkpoint: GEMM phase stamps, full GPU suite + smoke on the default (native) allocator,
# GPT bench native vs caching allocator, BERT (op-granular static program) and ResNet benches.
OUT=gpurun_out/${1:-r4e}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6; if fatal $rc; then exit $rc; fi; }
step stamps 200 python -u scripts/gemm_stamps.py
step tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_caching 300 env PRA_ALLOCATOR=caching python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
