#!/bin/bash
# Round 5: derivative-saving GELU epilogue + multiply-by-z dgrad, GPT / BERT shapes; GPT bench A/B.
OUT=gpurun_out/${1:-r5a}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 12; if fatal $rc; then exit $rc; fi; }
step mlp_gpt 200 python scripts/gemm_mlp_bench.py
step mlp_bert 200 python scripts/gemm_mlp_bench.py --bert
step bench_new 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_MLP_SAVE_D=0 step bench_old 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bench_new2 300 python bench.py --gpus 1 --steps 20 --warmup 5
exit 0
