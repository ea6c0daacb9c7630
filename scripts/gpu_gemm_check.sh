#!/bin/bash
# GEMM change check: numerics tests, per-shape table vs hipBLASLt, GPT bench x2.
OUT=gpurun_out/${1:-gemm_check}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 2 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_conv_kxk.py -x -q --timeout 120 --timeout-method thread
step gemm 200 python scripts/gemm_lds_bench.py
step bench_a 200 python bench.py --steps 20 --warmup 5
step bench_b 200 python bench.py --steps 20 --warmup 5
exit 0
