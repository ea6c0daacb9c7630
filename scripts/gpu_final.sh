#!/bin/bash
# End-of-session check: full GPU suite, driver bench command, GPT kernel profile, ResNet50 / BERT benches.
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step gemm 300 python scripts/gemm_lds_bench.py
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step fa 120 python -m scripts.fa_one 16 16 1024 128 1 50
exit 0
