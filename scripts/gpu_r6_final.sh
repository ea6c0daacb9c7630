#!/bin/bash
# Round 6 end: full GPU suite, smoke, driver bench command, GPT / ResNet / BERT benches and
# steady-state rocprofv3 kernel tables for all three.
OUT=gpurun_out/${1:-r6_final}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step gpt_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 4 --warmup 3
python scripts/trace_window.py $OUT/gpt_prof/gpt_kernel_trace.csv adamw_mt 3 45 > $OUT/gpt_table.md 2>&1; head -3 $OUT/gpt_table.md
step rn_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/rn_prof -o rn -- python bench.py --model resnet50 --steps 5 --warmup 3
python scripts/trace_window.py $OUT/rn_prof/rn_kernel_trace.csv momentum_mt 4 50 > $OUT/rn_table.md 2>&1; head -3 $OUT/rn_table.md
step bert_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/bert_prof -o bert -- python bench.py --model bert-base --steps 5 --warmup 3
python scripts/trace_window.py $OUT/bert_prof/bert_kernel_trace.csv adamw_mt 4 50 > $OUT/bert_table.md 2>&1; head -3 $OUT/bert_table.md
exit 0
