#!/bin/bash
# TN GEMMs with <= 128 rows on 128-row tiles: GEMM tests, full suite, ResNet A/B
OUT=gpurun_out/${1:-r3y}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step gemm 300 python -u -m pytest tests/test_gemm_lds_gpu.py -x -q --timeout 120 --timeout-method thread -k "narrow or layouts or beta"
step tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step rn_on 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_GEMM_NARROW=0 step rn_off 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_on2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step smoke 200 python __graft_entry__.py smoke
exit 0
