#!/bin/bash
# Round 5: channel-stationary BN apply kernels (coefficients in registers) -- tests + ResNet A/B.
OUT=gpurun_out/${1:-r5af}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_bn_dgrad_fuse.py tests/test_conv_bn_stats_gpu.py tests/test_grad_accum_gpu.py tests/test_resnet_aux.py -k "bn or batch or resnet or conv or residual or grad" -m gpu -x -q --timeout 120 --timeout-method thread
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_BN_APPLY_GENERIC=1 step rn_old 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_BN_APPLY_GENERIC=1 step rn_old2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_prof 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/rn_prof -o rn -- python bench.py --model resnet50 --steps 6 --warmup 4
python scripts/trace_window.py $OUT/rn_prof/rn_kernel_trace.csv momentum_mt 4 45 > $OUT/rn_table.md 2>&1; head -24 $OUT/rn_table.md
exit 0
