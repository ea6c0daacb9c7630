#!/bin/bash
# Static gradient-sum fusion (residual partial folded into the Linear / MLP dgrad): tests + BERT A/B.
OUT=gpurun_out/${1:-r4t}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_static.py tests/test_bert_gpu.py tests/test_kernels_gpu.py
step bert 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_prof 300 rocprofv3 --kernel-trace -d $OUT/bert_prof -o bert -- python bench.py --model bert-base --steps 20 --warmup 3
step bert2 300 python bench.py --model bert-base --steps 30 --warmup 5
exit 0
