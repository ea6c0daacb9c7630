#!/bin/bash
# Round 5: query-split (two waves per SIMD) head_dim-128 dK/dV kernel: numerics + A/B.
OUT=gpurun_out/${1:-r5h}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_flash_ext.py -x -q --timeout 120 --timeout-method thread -k "flash or attn or qkv"
step fa_qs 120 python -m scripts.fa_one 16 16 1024 128 1 50
PRA_FA_DKDV_QS=0 step fa_old 120 python -m scripts.fa_one 16 16 1024 128 1 50
step fa_qs_nc 120 python -m scripts.fa_one 8 16 2048 128 0 20
PRA_FA_DKDV_QS=0 step fa_old_nc 120 python -m scripts.fa_one 8 16 2048 128 0 20
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_FA_DKDV_QS=0 step gpt_old 300 python bench.py --gpus 1 --steps 20 --warmup 5

step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_prof 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/rn_prof -o rn -- python bench.py --model resnet50 --steps 6 --warmup 4
python scripts/trace_window.py $(ls $OUT/rn_prof/*/rn_kernel_trace.csv $OUT/rn_prof/rn_kernel_trace.csv 2>/dev/null | head -1) momentum_mt 4 45 > $OUT/rn_table.md 2>&1; head -50 $OUT/rn_table.md
exit 0
