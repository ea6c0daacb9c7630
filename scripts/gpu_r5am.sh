#!/bin/bash
# Round 5: max pool with 32-bit lane index math -- pool tests, kernel probe, ResNet bench.
OUT=gpurun_out/${1:-r5am}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pool_gpu.py tests/test_conv_kxk.py -m gpu
PYTHONPATH=. step probe 120 python scripts/pool_probe.py
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
exit 0
