#!/bin/bash
# BERT: short-K dgrad policy variants + per-kernel tables (rocprofv3) of policy on / off.
OUT=gpurun_out/${1:-r4o}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-140; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_lds_gpu.py -k "auto_policy or mlp_gelu or dgelu" tests/test_kernels_gpu.py tests/test_bert_gpu.py
step nomlp 300 env PRA_MLP_DGELU_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
step off 300 env PRA_GEMM_NT_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
step nomlp2 300 env PRA_MLP_DGELU_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
step off2 300 env PRA_GEMM_NT_SHORTK=0 python bench.py --model bert-base --steps 30 --warmup 5
step prof_on 300 rocprofv3 --kernel-trace -d $OUT/prof_on -o on -- python bench.py --model bert-base --steps 20 --warmup 3
exit 0
