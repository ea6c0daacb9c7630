#!/bin/bash
OUT=gpurun_out/${1:-r3q}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gemmbert 300 python scripts/gemm_lds_bench.py --bert
step rnprof 300 rocprofv3 --kernel-trace --stats -d $OUT/rnprof -o rn --output-format csv -- python3 bench.py --model resnet50 --steps 5 --warmup 2
exit 0
