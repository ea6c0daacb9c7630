#!/bin/bash
# TS default: GEMM GPU tests, GPT bench, GPT A/B vs the W8 baseline, BERT bench.
OUT=gpurun_out/${1:-r4h}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4; if fatal $rc; then exit $rc; fi; }
step mha3 200 python -u scripts/debug_mha3.py
step gemmtests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_lds_gpu.py tests/test_kernels_gpu.py
step gpt_ts 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_w8 300 env PRA_GEMM_W4=0 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_dgelu 300 env PRA_MLP_DGELU_EPI=1 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_mfma 300 env PRA_MLP_DGELU_EPI=1 PRA_GEMM=mfma python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_ts2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
exit 0
