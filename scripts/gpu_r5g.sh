#!/bin/bash
# Round 5: GPT / BERT step A/B of the derivative-saving MLP (PRA_MLP_SAVE_D), interleaved.
OUT=gpurun_out/${1:-r5g}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
for r in 1 2; do
step gpt_new_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_MLP_SAVE_D=0 step gpt_old_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert_new_$r 300 python bench.py --model bert-base --steps 20 --warmup 5
PRA_MLP_SAVE_D=0 step bert_old_$r 300 python bench.py --model bert-base --steps 20 --warmup 5
done
exit 0
