#!/bin/bash
# Round-3 re-entry check on the committed tree: full GPU suite, smoke, driver-style GPT bench,
# BERT / ResNet benches, FA probe, GEMM table, rocprofv3 kernel stats of GPT, BERT and ResNet.
OUT=gpurun_out/${1:-r3f}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 4 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step fa 200 python scripts/fa_probe.py
step gemm 300 python scripts/gemm_lds_bench.py
step gptprof 300 rocprofv3 --kernel-trace --stats -d $OUT/gptprof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
step bertprof 300 rocprofv3 --kernel-trace --stats -d $OUT/bertprof -o bert --output-format csv -- python3 bench.py --model bert-base --steps 5 --warmup 2
step rnprof 300 rocprofv3 --kernel-trace --stats -d $OUT/rnprof -o rn --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 2
exit 0
