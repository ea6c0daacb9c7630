#!/bin/bash
# Round 5: add+dropout+LayerNorm backward workgroup count (PRA_ADL_NBLK, default 768) -- BERT sweep,
# same box.
OUT=gpurun_out/${1:-r5ap}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step bert_768 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_ADL_NBLK=512 step bert_512 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_ADL_NBLK=1024 step bert_1024 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_ADL_NBLK=1536 step bert_1536 300 python bench.py --model bert-base --steps 30 --warmup 5
PRA_ADL_NBLK=2048 step bert_2048 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_768b 300 python bench.py --model bert-base --steps 30 --warmup 5
exit 0
