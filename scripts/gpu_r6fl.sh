#!/bin/bash
# Round 6: long-K x·W on the persistent kernel (PRA_GEMM_FWD_LONGK_PTS) A/B on the GPT step.
OUT=gpurun_out/${1:-r6fl}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-180; if fatal $rc; then exit $rc; fi; }
step t 600 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step b1 300 env PRA_GEMM_FWD_LONGK_PTS=1 python bench.py --steps 20 --warmup 5
step b0 300 env PRA_GEMM_FWD_LONGK_PTS=0 python bench.py --steps 20 --warmup 5
step b1b 300 env PRA_GEMM_FWD_LONGK_PTS=1 python bench.py --steps 20 --warmup 5
step b0b 300 env PRA_GEMM_FWD_LONGK_PTS=0 python bench.py --steps 20 --warmup 5
exit 0
