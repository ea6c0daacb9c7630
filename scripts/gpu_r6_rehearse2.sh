#!/bin/bash
# Round 6: 4-rank rehearsal on one MI355X (gloo): smaller model first, then 1.3B with a tick file
# so a slow (host-copy bound) run is not mistaken for a hang; tracebacks dumped on timeout.
OUT=gpurun_out/${1:-r6_rehearse2}
mkdir -p $OUT
export TMPDIR=/tmp
( for i in $(seq 1 60); do date +%T >> $OUT/ticks.log; sleep 20; done ) &
TICK=$!
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "Gloo\|socket.cpp" | tail -n 4 | cut -c1-300; if fatal $rc; then kill $TICK; exit $rc; fi; }
step w4s 300 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=280 PRA_BENCH_TRACE=1 python bench.py --gpus 4 --steps 2 --warmup 1 --model gpt3-125m --micro-batch 4
step w4 560 env PRA_DIST_BACKEND=gloo PRA_BENCH_TIMEOUT=540 PRA_BENCH_TRACE=1 python bench.py --gpus 4 --steps 1 --warmup 1 --micro-batch 4
kill $TICK
exit 0
