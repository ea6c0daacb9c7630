#!/bin/bash
# BERT step with the dQ kernel launch shapes (PRA_FA_DQ), interleaved.
OUT=gpurun_out/${1:-r4an}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for v in 8x3 4x3 4x4 8x2; do
    step bert_${v}_$i 300 env PRA_FA_DQ=$v python bench.py --model bert-base --steps 40 --warmup 5
  done
done
step gpt_4x4 300 env PRA_FA_DQ=4x4 python bench.py --steps 12 --warmup 4
step gpt_8x3 300 env PRA_FA_DQ=8x3 python bench.py --steps 12 --warmup 4
exit 0
