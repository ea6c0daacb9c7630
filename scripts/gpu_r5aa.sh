#!/bin/bash
# Round 5: QKV + out-projection weight gradients in one grouped launch (GPT A/B).
OUT=gpurun_out/${1:-r5aa}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_flash_ext.py tests/test_opt_overlap_gpu.py tests/test_tp_fused.py tests/test_models_io.py -m gpu -x -q --timeout 120 --timeout-method thread
step gpt 300 python bench.py --steps 10 --warmup 3
PRA_WGRAD_PAIR=0 step gpt_old 300 python bench.py --steps 10 --warmup 3
step gpt2 300 python bench.py --steps 10 --warmup 3
PRA_WGRAD_PAIR=0 step gpt_old2 300 python bench.py --steps 10 --warmup 3
exit 0
