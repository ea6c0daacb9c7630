#!/bin/bash
# Round 5: grid-stride attention delta kernel (tests + GPT A/B against the previous build's number).
OUT=gpurun_out/${1:-r5ak}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_flash_ext.py tests/test_kernels_gpu.py -k "flash or delta or attn" -m gpu -x -q --timeout 120 --timeout-method thread
step gpt_prof 500 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 4 --warmup 3
python scripts/trace_window.py $OUT/gpt_prof/gpt_kernel_trace.csv adamw_mt 3 45 > $OUT/gpt_table.md 2>&1; grep -E "kernel time|attn_delta" $OUT/gpt_table.md
exit 0
