#!/bin/bash
# Round 6 batch O: GPU tier + smoke + GPT bench + end-of-round kernel table.
OUT=gpurun_out/${1:-r6o}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step gputests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --steps 20 --warmup 5
step gpt_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 4 --warmup 3
python scripts/trace_window.py $OUT/gpt_prof/gpt_kernel_trace.csv adamw_mt 3 45 > $OUT/gpt_table.md 2>&1; head -24 $OUT/gpt_table.md
exit 0
