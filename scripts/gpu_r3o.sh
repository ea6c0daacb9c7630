#!/bin/bash
OUT=gpurun_out/${1:-r3o}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_lds_gpu.py tests/test_bert_gpu.py -m gpu -q --timeout 200 --timeout-method thread
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step bert2 300 python bench.py --model bert-base --steps 20 --warmup 5
exit 0
