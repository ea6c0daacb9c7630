#!/bin/bash
# MHA flash-ext debug, BERT static direct-grad A/B (graph and op by op), GPT bench x2.
OUT=gpurun_out/${1:-r4f}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6; if fatal $rc; then exit $rc; fi; }
step stamps 200 python -u scripts/gemm_stamps.py
step mha 200 python -u scripts/debug_mha.py
step bert_direct 300 python bench.py --model bert-base --steps 20 --warmup 5
step bert_vjp 300 env PRA_STATIC_DIRECT_GRAD=0 python bench.py --model bert-base --steps 20 --warmup 5
step bert_direct_nog 300 python bench.py --model bert-base --steps 10 --warmup 3 --no-graph
step bert_vjp_nog 300 env PRA_STATIC_DIRECT_GRAD=0 python bench.py --model bert-base --steps 10 --warmup 3 --no-graph
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
exit 0
