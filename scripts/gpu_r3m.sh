#!/bin/bash
OUT=gpurun_out/${1:-r3m}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 500 python -u -m pytest tests/test_native_allocator.py tests/test_gemm_lds_gpu.py tests/test_grad_accum_gpu.py -m gpu -q --timeout 200 --timeout-method thread
step bert_alloc 300 env PRA_ALLOCATOR=auto_growth python bench.py --model bert-base --steps 20 --warmup 5
step bert_base 300 python bench.py --model bert-base --steps 20 --warmup 5
step rn_alloc 300 env PRA_ALLOCATOR=auto_growth python bench.py --model resnet50 --steps 20 --warmup 5
step rn_base 300 python bench.py --model resnet50 --steps 20 --warmup 5
step bert_alloc2 300 env PRA_ALLOCATOR=auto_growth python bench.py --model bert-base --steps 20 --warmup 5
exit 0
