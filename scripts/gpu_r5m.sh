#!/bin/bash
# Round 5: dy·Wᵀ in-tree up to K = 3072 (PRA_GEMM_NT_MAXK) A/B on GPT and BERT.
OUT=gpurun_out/${1:-r5m}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_gemm_lds_gpu.py -x -q --timeout 120 --timeout-method thread -k "auto_policy or mlp or many_tiles"
for r in 1 2; do
step gpt_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_GEMM_NT_MAXK=1024 step gpt_old_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert_$r 300 python bench.py --model bert-base --steps 20 --warmup 5
PRA_GEMM_NT_MAXK=1024 step bert_old_$r 300 python bench.py --model bert-base --steps 20 --warmup 5
done
exit 0
