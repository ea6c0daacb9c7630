#!/bin/bash
# BERT with / without the committed TunableOp solutions (GPT + BERT shapes), interleaved; GPT check.
OUT=gpurun_out/${1:-r4ah}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  step bert_tuned_$i 300 python bench.py --model bert-base --steps 40 --warmup 5
  step bert_untuned_$i 300 python bench.py --model bert-base --steps 40 --warmup 5 --no-tuned-gemms
done
step gpt_tuned 300 python bench.py --steps 20 --warmup 5
exit 0
