#!/bin/bash
# Round 5: multi-lane split-K reduce (small outputs, many splits): tests + ResNet / BERT / GPT A/B.
OUT=gpurun_out/${1:-r5ai}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_conv_kxk.py tests/test_kernels_gpu.py tests/test_grad_accum_gpu.py tests/test_conv1x1.py -m gpu -x -q --timeout 120 --timeout-method thread
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_SPLITK_GMAX=1 step rn_old 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_SPLITK_GMAX=1 step rn_old2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step bert 300 python bench.py --model bert --steps 20 --warmup 5
PRA_SPLITK_GMAX=1 step bert_old 300 python bench.py --model bert --steps 20 --warmup 5
step bert2 300 python bench.py --model bert --steps 20 --warmup 5
PRA_SPLITK_GMAX=1 step bert_old2 300 python bench.py --model bert --steps 20 --warmup 5
exit 0
