#!/bin/bash
# TunableOp GEMM solutions (paddle_ray_amd/tuning/gemm_gfx950.csv) A/B, interleaved, + kernel table.
OUT=gpurun_out/${1:-r4af}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  step tuned_$i 300 python bench.py --steps 20 --warmup 5
  step untuned_$i 300 python bench.py --steps 20 --warmup 5 --no-tuned-gemms
done
step prof 400 rocprofv3 --kernel-trace -d $OUT/prof -o gpt -- python bench.py --steps 10 --warmup 3
exit 0
