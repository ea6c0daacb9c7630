#!/bin/bash
# Round 5: split-K reduce lanes per output quad (PRA_SPLITK_GMAX, default 64) on BERT -- same box.
OUT=gpurun_out/${1:-r5aq}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step bert_64 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_SPLITK_GMAX=1 step bert_1 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_SPLITK_GMAX=8 step bert_8 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_SPLITK_GMAX=16 step bert_16 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_64b 300 python bench.py --model bert-base --steps 30 --warmup 5
exit 0
