#!/bin/bash
# Round-3 checks: new GPU tests (flash extensions, jit graph semantics, custom ops), then the
# W4 GEMM comparison.
OUT=gpurun_out/${1:-r3a}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 25 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step newtests 400 python -u -m pytest tests/test_flash_ext.py tests/test_jit.py tests/test_cpp_extension.py -m gpu -v --timeout 120 --timeout-method thread
step w4 300 python scripts/gemm_lds_bench.py --w4
step fused8 120 python scripts/gemm_lds_bench.py --fused
step fused4 120 python scripts/gemm_lds_bench.py --fused --w4
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step bertprof 300 rocprofv3 --kernel-trace --stats -d $OUT/bprof -o bert --output-format csv -- python3 bench.py --model bert-base --steps 5 --warmup 2
step gpt 300 python bench.py --steps 20 --warmup 5
exit 0
