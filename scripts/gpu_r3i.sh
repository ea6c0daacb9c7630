#!/bin/bash
# BERT fused MLP + GEMM split policy; ResNet 1x1 conv + BN-stats fusion (A/B) and HIP-graph step.
OUT=gpurun_out/${1:-r3i}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_conv_bn_stats_gpu.py tests/test_resnet_unit.py -m gpu -q -x --timeout 120 --timeout-method thread

step rn_new 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_old 300 env PRA_CONV1X1_STATS=0 python bench.py --model resnet50 --steps 20 --warmup 5

step rn_new2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_old2 300 env PRA_CONV1X1_STATS=0 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
