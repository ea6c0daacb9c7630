#!/bin/bash
# ResNet50 A/B: 1x1 conv via hipBLASLt GEMM (default) vs MIOpen; + profile of the default.
OUT=gpurun_out/${1:-rnab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 2 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "conv1x1 or resnet"
step gemm 300 python bench.py --model resnet50 --steps 10 --warmup 3
PRA_CONV1X1_GEMM=0 step miopen 300 python bench.py --model resnet50 --steps 10 --warmup 3
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o rn --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2
exit 0
