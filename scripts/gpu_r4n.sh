#!/bin/bash
# Short-K dy·Wᵀ on the persistent in-tree kernel (+ fused dGELU epilogue in BERT's MLP) and the
# static add+dropout+LN grad without the zero fill: GPU tests, then BERT A/B (policy on / off).
OUT=gpurun_out/${1:-r4n}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_lds_gpu.py tests/test_kernels_gpu.py tests/test_bert_gpu.py tests/test_static_gpu.py
step bert_on 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_off 300 env PRA_GEMM_NT_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
step bert_on2 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_off2 300 env PRA_GEMM_NT_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
exit 0
