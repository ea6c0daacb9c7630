#!/bin/bash
# Same-box A/B: static gradient-sum fold, flash bias partials (BERT), interleaved.
OUT=gpurun_out/${1:-r4u}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  step on_$i 300 python bench.py --model bert-base --steps 40 --warmup 5
  step nofold_$i 300 env PRA_STATIC_GRAD_FOLD=0 python bench.py --model bert-base --steps 40 --warmup 5
  step none_$i 300 env PRA_STATIC_GRAD_FOLD=0 PRA_FA_BIAS_PART=0 python bench.py --model bert-base --steps 40 --warmup 5
done
exit 0
