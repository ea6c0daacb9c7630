#!/bin/bash
# GPU kernel tests + smoke + GPT bench + GPT rocprofv3 kernel stats.
OUT=gpurun_out/${1:-ktb}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 10 --warmup 3
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 2 --warmup 1
exit 0
