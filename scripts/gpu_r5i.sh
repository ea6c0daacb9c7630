#!/bin/bash
# Round 5 checkpoint: full GPU suite, smoke, GPT bench + steady-state GPT kernel table.
OUT=gpurun_out/${1:-r5i}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python __graft_entry__.py smoke
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_prof 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 8 --warmup 3
python scripts/trace_window.py $(ls $OUT/gpt_prof/gpt_kernel_trace.csv $OUT/gpt_prof/*/gpt_kernel_trace.csv 2>/dev/null | head -1) adamw_mt 4 40 > $OUT/gpt_table.md 2>&1; head -45 $OUT/gpt_table.md
exit 0
