#!/bin/bash
# Round 6 batch I: GPT bench A/B of the side-stream gradient zeroing and the AdamW unroll.
OUT=gpurun_out/${1:-r6i}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step base 300 python bench.py --steps 20 --warmup 5
PRA_ZERO_SIDE=0 step off 300 python bench.py --steps 20 --warmup 5
step base2 300 python bench.py --steps 20 --warmup 5
PRA_ZERO_SIDE=0 step off2 300 python bench.py --steps 20 --warmup 5
step beta 200 python scripts/r6_beta_probe.py
exit 0
