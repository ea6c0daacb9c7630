#!/bin/bash
# final check of the committed tree: GPU suite, smoke, the three benches
OUT=gpurun_out/${1:-r3final}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rnops 300 python bench.py --model resnet50 --steps 3 --warmup 2 --profile-dir $OUT/rnops
exit 0
