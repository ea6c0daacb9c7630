#!/bin/bash
# Round 5: strided dgrad phase tests (opt-in path) + BN-dgrad fusion tests + GEMM suite.
OUT=gpurun_out/${1:-r5x}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_conv_kxk.py tests/test_bn_dgrad_fuse.py tests/test_gemm_lds_gpu.py tests/test_resnet_aux.py -m gpu -x -q --timeout 120 --timeout-method thread
exit 0
