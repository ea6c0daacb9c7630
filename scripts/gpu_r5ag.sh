#!/bin/bash
# Round 5: BERT kernel table (end of round).
OUT=gpurun_out/${1:-r5ag}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step bert_prof 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/bert_prof -o bert -- python bench.py --model bert --steps 6 --warmup 4
python scripts/trace_window.py $OUT/bert_prof/bert_kernel_trace.csv adamw_mt 4 45 > $OUT/bert_table.md 2>&1; head -40 $OUT/bert_table.md
exit 0
