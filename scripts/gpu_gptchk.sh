#!/bin/bash
OUT=gpurun_out/${1:-gptchk}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step fa 200 python scripts/fa_probe.py
step gpt 300 python bench.py --steps 10 --warmup 3
step gptprof 300 rocprofv3 --kernel-trace --stats -d $OUT/gptprof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
step gpt2 300 python bench.py --steps 10 --warmup 3
exit 0
