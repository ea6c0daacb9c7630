#!/bin/bash
# BERT bench after dropping the hipBLASLt routing for split forwards, then a GPT kernel trace
OUT=gpurun_out/${1:-r3r}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gptprof 400 rocprofv3 --kernel-trace --stats -d $OUT/gptprof -o gpt --output-format csv -- python3 bench.py --gpus 1 --steps 4 --warmup 2
exit 0
