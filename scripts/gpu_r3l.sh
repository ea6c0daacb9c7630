#!/bin/bash
# Native allocator with graph pools: tests, BERT (HIP-graph static executor) and ResNet benches.
OUT=gpurun_out/${1:-r3l}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 500 python -u -m pytest tests/test_native_allocator.py -m gpu -q -x --timeout 200 --timeout-method thread
step bert_alloc 300 env PRA_ALLOCATOR=auto_growth python bench.py --model bert-base --steps 20 --warmup 5
step rn_alloc 300 env PRA_ALLOCATOR=auto_growth python bench.py --model resnet50 --steps 20 --warmup 5
step suite_alloc 900 env PRA_ALLOCATOR=auto_growth python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
exit 0
