#!/bin/bash
# Round 6 batch K: GEMM GPU tests with the dynamic persistent tile order; GPT bench.
OUT=gpurun_out/${1:-r6k}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step gemmtests 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or Gemm or linear or mlp or Linear"
step bench 300 python bench.py --steps 20 --warmup 5
PRA_PTS_DYN=0 step bench_static 300 python bench.py --steps 20 --warmup 5
exit 0
