#!/bin/bash
# ResNet-50: MIOpen exhaustive find for the convolutions it still runs, A/B interleaved.
OUT=gpurun_out/${1:-r4ai}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  step find_$i 400 python bench.py --model resnet50 --steps 20 --warmup 5
  step heur_$i 400 env PRA_MIOPEN_FIND=0 python bench.py --model resnet50 --steps 20 --warmup 5
done
exit 0
