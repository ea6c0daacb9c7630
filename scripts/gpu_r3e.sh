#!/bin/bash
# GEMM configs (numerics + A/B incl. MUBUF DMA), conv+BN-statistics fusion, ZeRO-3 fix,
# BERT keep-bits A/B, ResNet with/without conv-stats fusion.
OUT=gpurun_out/${1:-r3e}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 8 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_conv_bn_stats_gpu.py tests/test_zero3_gpu.py tests/test_resnet_unit.py -m gpu -q --timeout 120 --timeout-method thread
step gemmab 400 python scripts/gemm_lds_bench.py --w4
step bert_bits 300 python bench.py --model bert-base --steps 20 --warmup 5
step bert_nobits 300 env PRA_FA_DROP_BITS=0 python bench.py --model bert-base --steps 20 --warmup 5
step resnet_stats 300 python bench.py --model resnet50 --steps 10 --warmup 3
step resnet_nostats 300 env PRA_CONV_BN_STATS=0 python bench.py --model resnet50 --steps 10 --warmup 3
exit 0
