#!/bin/bash
# Full GPU check: GPU tests, FA probe, GPT bench, rocprofv3 kernel stats.
# Stops at the first fault / timeout (no further GPU steps after one).
OUT=gpurun_out/${1:-round}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 4 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 600 python -m pytest tests -m gpu -x -q
step fa 200 python scripts/fa_probe.py
step bench 500 python bench.py --steps 10 --warmup 3
step prof 500 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 3 --warmup 2
exit 0
