#!/bin/bash
# GPU check: GPU tests, smoke, GPT bench, ResNet50 bench. Stops at the first fault/timeout.
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 4 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 10 --warmup 3
step resnet 400 python bench.py --model resnet50 --steps 10 --warmup 3
exit 0
