#!/bin/bash
# Extended flash attention: numerics tests, BERT-shape probe, BERT bench.
OUT=gpurun_out/${1:-faext}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 8 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_flash_ext.py tests/test_kernels_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step probe 200 python scripts/fa_ext_probe.py
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
exit 0
