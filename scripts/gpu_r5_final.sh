#!/bin/bash
# Round 5 end: full GPU suite, smoke, driver bench command, GPT / ResNet / BERT benches.
OUT=gpurun_out/${1:-r5_final}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
exit 0
