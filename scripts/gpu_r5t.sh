#!/bin/bash
# Round 5: AdamW body variants; ResNet 56x56 1x1 forwards on the in-tree stats conv (A/B).
OUT=gpurun_out/${1:-r5t}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
for v in 0 1 2 3 0 1 2; do PRA_ADAMW_V8=$v step adamw_v$v 120 python scripts/adamw_bench.py; done
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -k "resnet or adamw" -x -q --timeout 120 --timeout-method thread
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_CONV1X1_STATS_ALL=1 step rn_all 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_CONV1X1_STATS_ALL=1 step rn_all2 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
