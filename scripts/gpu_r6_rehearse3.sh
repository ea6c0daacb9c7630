#!/bin/bash
# Round 6: which part stalls the 4-rank gloo rehearsal on one GPU: sharding stage 2 vs 1 vs 3.
OUT=gpurun_out/${1:-r6_rehearse3}
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 40); do date +%T >> $OUT/ticks.log; sleep 20; done ) &
TICK=$!
fatal() { case $1 in 137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "Gloo\|socket.cpp" | tail -n 2 | cut -c1-200; if fatal $rc; then kill $TICK; exit $rc; fi; }
step os_g 170 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=150 PRA_BENCH_TRACE=100 python bench.py --gpus 4 --steps 2 --warmup 1 --model gpt3-125m --micro-batch 4 --level os_g
step os 170 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=150 PRA_BENCH_TRACE=100 python bench.py --gpus 4 --steps 2 --warmup 1 --model gpt3-125m --micro-batch 4 --level os
step w3 170 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=150 PRA_BENCH_TRACE=100 python bench.py --gpus 3 --steps 2 --warmup 1 --model gpt3-125m --micro-batch 4
kill $TICK
exit 0
