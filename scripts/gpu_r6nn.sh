#!/bin/bash
# Round 6: narrow dy·Wᵀ (N <= 1024, K <= 4096) in-tree (PRA_GEMM_NT_NARROWN) A/B on BERT / ResNet / GPT.
OUT=gpurun_out/${1:-r6nn}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step gemmtests 600 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step bert1 300 env PRA_GEMM_NT_NARROWN=1024 python bench.py --model bert-base --steps 20 --warmup 5
step bert0 300 env PRA_GEMM_NT_NARROWN=0 python bench.py --model bert-base --steps 20 --warmup 5
step bert1b 300 env PRA_GEMM_NT_NARROWN=1024 python bench.py --model bert-base --steps 20 --warmup 5
step bert0b 300 env PRA_GEMM_NT_NARROWN=0 python bench.py --model bert-base --steps 20 --warmup 5
step rn1 300 env PRA_GEMM_NT_NARROWN=1024 python bench.py --model resnet50 --steps 20 --warmup 5
step rn0 300 env PRA_GEMM_NT_NARROWN=0 python bench.py --model resnet50 --steps 20 --warmup 5
step rn1b 300 env PRA_GEMM_NT_NARROWN=1024 python bench.py --model resnet50 --steps 20 --warmup 5
step rn0b 300 env PRA_GEMM_NT_NARROWN=0 python bench.py --model resnet50 --steps 20 --warmup 5
step gpt1 300 env PRA_GEMM_NT_NARROWN=1024 python bench.py --steps 20 --warmup 5
exit 0
