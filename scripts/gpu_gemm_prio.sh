#!/bin/bash
# GEMM priority-mode A/B: per-shape ratio vs hipBLASLt and the GPT step, PRA_GEMM_PRIO=0 vs 1.
OUT=gpurun_out/${1:-gemm_prio}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 19 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step test 200 python -u -m pytest tests/test_gemm_lds_gpu.py -x -q --timeout 120 --timeout-method thread
step g0 200 env PRA_GEMM=mfma PRA_GEMM_PRIO=0 python scripts/gemm_lds_bench.py
step g1 200 env PRA_GEMM=mfma PRA_GEMM_PRIO=1 python scripts/gemm_lds_bench.py
step b0 200 env PRA_GEMM_PRIO=0 python bench.py --steps 20 --warmup 5
step b1 200 env PRA_GEMM_PRIO=1 python bench.py --steps 20 --warmup 5
step b0r 200 env PRA_GEMM_PRIO=0 python bench.py --steps 20 --warmup 5
step b1r 200 env PRA_GEMM_PRIO=1 python bench.py --steps 20 --warmup 5
exit 0
