#!/bin/bash
# Round 6: channels-last NHWC KxK filters (PRA_CONV_CL_WEIGHTS): conv tests, ResNet-50 A/B + kernel table.
OUT=gpurun_out/${1:-r6cl}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "^[WE]2026" | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step convtests 600 python -u -m pytest tests/test_conv_kxk.py tests/test_conv1x1.py tests/test_conv_bn_stats_gpu.py tests/test_resnet_unit.py tests/test_bn_dgrad_fuse.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step rn1 300 env PRA_CONV_CL_WEIGHTS=1 python bench.py --model resnet50 --steps 20 --warmup 5
step rn0 300 env PRA_CONV_CL_WEIGHTS=0 python bench.py --model resnet50 --steps 20 --warmup 5
step rn1b 300 env PRA_CONV_CL_WEIGHTS=1 python bench.py --model resnet50 --steps 20 --warmup 5
step rn0b 300 env PRA_CONV_CL_WEIGHTS=0 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/rn_prof -o rn -- python bench.py --model resnet50 --steps 5 --warmup 3
python scripts/trace_window.py $OUT/rn_prof/rn_kernel_trace.csv momentum_mt 4 50 > $OUT/rn_table.md 2>&1; head -30 $OUT/rn_table.md
exit 0
