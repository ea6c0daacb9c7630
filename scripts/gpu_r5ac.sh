#!/bin/bash
# Round 5: BERT after the LinearFn signature change (static fn-op predicate), static GPU tests.
OUT=gpurun_out/${1:-r5ac}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_static.py tests/test_static_ir.py tests/test_bert.py tests/test_bert_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step bert 300 python bench.py --model bert --steps 20 --warmup 5
step bert2 300 python bench.py --model bert --steps 20 --warmup 5
exit 0
