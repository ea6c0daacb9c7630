#!/bin/bash
# Quick iteration: one GPU test file (optional), GPT bench (+ per-op stack tables), rocprofv3 kernel stats.
# usage: gpu_quick.sh OUT [test-file-or-none] [prof: 0|1]
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
if [ "${2:-none}" != none ]; then
  step tests 300 python -u -m pytest $2 -m gpu -x -q --timeout 120 --timeout-method thread
fi
step fa 120 python -m scripts.fa_one 16 16 1024 128 1 50
step bench 300 python bench.py --steps 20 --warmup 5 --profile-dir $OUT/ops
if [ "${3:-1}" = 1 ]; then
  step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
fi
exit 0
