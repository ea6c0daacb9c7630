#!/bin/bash
# Round 6 batch A: flash causal prologue overlap + sigmoid-form tanh-GELU epilogue.
OUT=gpurun_out/${1:-r6a}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 12 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step fa_causal 120 python scripts/fa_probe.py --B 16 --S 1024 --H 16 --D 128 --causal 1
step fa_nc 120 python scripts/fa_probe.py --B 8 --S 2048 --H 16 --D 128 --causal 0 --check 0
step gemm 300 python scripts/r6_gemm_probe.py
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_lds_gpu.py tests/test_flash_ext.py tests/test_kernels_gpu.py -m gpu
step bench 240 python bench.py --steps 10 --warmup 3
exit 0
