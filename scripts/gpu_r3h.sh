#!/bin/bash
# BERT with the fused MLP + GEMM split policy; ResNet eager vs HIP-graph step.
OUT=gpurun_out/${1:-r3h}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_bert_gpu.py tests/test_gemm_lds_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step rngraph 400 python scripts/resnet_graph.py
exit 0
