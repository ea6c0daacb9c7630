#!/bin/bash
# Round 6: the multi-rank bench path rehearsed on ONE MI355X (gloo collectives, ranks share the
# device; RCCL refuses two ranks per GPU): world 2 at the bench micro-batch, world 4 at mb 4.
OUT=gpurun_out/${1:-r6_rehearse}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4 | cut -c1-400; if fatal $rc; then exit $rc; fi; }
step w2 400 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=380 python bench.py --gpus 2 --steps 2 --warmup 1
step w4 400 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=380 python bench.py --gpus 4 --steps 2 --warmup 1 --micro-batch 4
exit 0
