#!/bin/bash
# Round 5: TN (weight-gradient) GEMMs on the W8 base config instead of W8T (fc1/fc2/head wgrads; the
# grouped QKV+out launch keeps W8T) -- GPT A/B.
OUT=gpurun_out/${1:-r5al}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step gpt 300 python bench.py --steps 10 --warmup 3
PRA_GEMM_W4=301989888 step gpt_w8 300 python bench.py --steps 10 --warmup 3
step gpt2 300 python bench.py --steps 10 --warmup 3
PRA_GEMM_W4=301989888 step gpt_w82 300 python bench.py --steps 10 --warmup 3
exit 0
