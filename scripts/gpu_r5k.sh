#!/bin/bash
# Round 5: persistent 4-wave fused GELU forward + bias-grad partials into b.grad; GEMM tests, GPT A/B.
OUT=gpurun_out/${1:-r5k}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
for r in 1 2; do
step gpt_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_MLP_MULZ_PTS=0 step gpt_ts_$r 300 python bench.py --gpus 1 --steps 20 --warmup 5
done
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
exit 0
