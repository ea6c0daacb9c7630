#!/bin/bash
OUT=gpurun_out/${1:-gemm}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gemm_lds_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -3 $OUT/tests.log
[ $rc -ne 0 ] && { grep -E "^E |Error" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/gemm_lds_bench.py > $OUT/bench.log 2>&1; rc=$?
tail -18 $OUT/bench.log
exit $rc
