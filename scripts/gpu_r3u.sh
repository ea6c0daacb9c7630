#!/bin/bash
# full GPU suite and the three benches with the native allocator (record_stream honoured)
OUT=gpurun_out/${1:-r3u}
mkdir -p $OUT
export TMPDIR=/tmp
export PRA_ALLOCATOR=auto_growth
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
unset PRA_ALLOCATOR
step gpt_torch 300 python bench.py --gpus 1 --steps 20 --warmup 5
step resnet_torch 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
