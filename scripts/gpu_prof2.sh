#!/bin/bash
# rocprofv3 kernel stats of the BERT and ResNet benches (+ GPT bench as a regression check).
OUT=gpurun_out/${1:-prof2}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step bertprof 300 rocprofv3 --kernel-trace --stats -d $OUT/bertprof -o bert --output-format csv -- python3 bench.py --model bert-base --steps 5 --warmup 2
step rnprof 300 rocprofv3 --kernel-trace --stats -d $OUT/rnprof -o rn --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 2
step gpt 300 python bench.py --steps 10 --warmup 3
exit 0
