#!/bin/bash
# Round 5: strided 3x3 dgrad as four sub-pixel phases on the implicit-GEMM kernel.
OUT=gpurun_out/${1:-r5u}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_conv_kxk.py tests/test_bn_dgrad_fuse.py tests/test_conv_bn_stats_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step probe 200 python scripts/strided_dgrad_probe.py
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_STRIDED_DGRAD=0 step rn_old 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
