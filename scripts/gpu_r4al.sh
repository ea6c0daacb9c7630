#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke, GPT bench (driver command), BERT bench.
OUT=gpurun_out/${1:-r4al}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step gputests 900 python -u -m pytest tests/ -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 40 --warmup 5
step bert2 300 python bench.py --model bert-base --steps 40 --warmup 5
exit 0
