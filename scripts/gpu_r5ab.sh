#!/bin/bash
# Round 5: GPT kernel table after the grouped weight gradients; BERT bench.
OUT=gpurun_out/${1:-r5ab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step gpt_prof 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 4 --warmup 3
python scripts/trace_window.py $OUT/gpt_prof/gpt_kernel_trace.csv adamw_mt 3 45 > $OUT/gpt_table.md 2>&1; head -40 $OUT/gpt_table.md
step bert 300 python bench.py --model bert --steps 20 --warmup 5
exit 0
