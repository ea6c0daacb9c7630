#!/bin/bash
# Round 5: conv filters (OHWI + flipped IHWO) from one forward launch
# -- BN / conv / ResNet GPU tests, then a same-box ResNet A/B (PRA_CONV_WPREP=0 = two launches).
OUT=gpurun_out/${1:-r5ao}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bn_dgrad_fuse.py tests/test_kernels_gpu.py tests/test_conv_kxk.py tests/test_grad_accum_gpu.py tests/test_resnet_aux.py
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_CONV_WPREP=0 step rn_two 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_CONV_WPREP=0 step rn_two2 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
