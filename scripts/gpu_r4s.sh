#!/bin/bash
OUT=gpurun_out/${1:-r4s}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_flash_ext.py tests/test_bert_gpu.py tests/test_static.py tests/test_gemm_lds_gpu.py
exit 0
