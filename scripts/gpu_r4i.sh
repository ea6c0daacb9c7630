#!/bin/bash
# Persistent TS GEMM: GEMM GPU tests, 15-shape table, GPT A/B (PTS on/off, dGELU epilogue), MHA debug.
OUT=gpurun_out/${1:-r4i}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 4; if fatal $rc; then exit $rc; fi; }
step gemmtests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_lds_gpu.py -k "PTS or TS"
step fatests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_flash_ext.py tests/test_kernels_gpu.py -k "flash or attn or fa_"
step faprobe 200 python -u scripts/fa_probe.py --causal 1 --check 1
step faext 200 python -u scripts/fa_ext_probe.py
step pts 400 python -u scripts/gemm_lds_bench.py --w4 --pts
step pts_bert 300 python -u scripts/gemm_lds_bench.py --w4 --pts --bert
step gpt_pts 300 env PRA_GEMM_PTS=7 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_nopts 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_dgelu 300 env PRA_GEMM_PTS=7 PRA_MLP_DGELU_EPI=1 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_mfma 300 env PRA_GEMM_PTS=7 PRA_MLP_DGELU_EPI=1 PRA_GEMM=mfma python bench.py --gpus 1 --steps 20 --warmup 5
step bert_pts 300 env PRA_GEMM_PTS=7 python bench.py --model bert-base --steps 20 --warmup 5
step mha3 200 python -u scripts/debug_mha3.py
step gemmall 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_lds_gpu.py tests/test_kernels_gpu.py
exit 0
