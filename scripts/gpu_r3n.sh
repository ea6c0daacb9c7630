#!/bin/bash
OUT=gpurun_out/${1:-r3n}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 500 python -u -m pytest tests/test_bert_gpu.py tests/test_jit_train_graph.py tests/test_static.py tests/test_static_ir.py tests/test_flash_ext.py -m gpu -q --timeout 200 --timeout-method thread
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step bertprof 300 rocprofv3 --kernel-trace --stats -d $OUT/bertprof -o bert --output-format csv -- python3 bench.py --model bert-base --steps 5 --warmup 2
exit 0
