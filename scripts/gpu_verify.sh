#!/bin/bash
# Round check on one MI355X: full GPU test suite, the driver's exact bench command, FA probe.
# Stops at the first fault / timeout (no further GPU steps after one).
OUT=gpurun_out/${1:-verify}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 500 python bench.py --gpus 1 --steps 20 --warmup 5
step fa 200 python -m scripts.fa_one 16 16 1024 128 1 50
exit 0
