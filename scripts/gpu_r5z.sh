#!/bin/bash
# Round 5: ResNet step under jit.to_static HIP-graph training capture (accumulate mode).
OUT=gpurun_out/${1:-r5z}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_jit_train_graph.py tests/test_native_allocator.py -m gpu -x -q --timeout 120 --timeout-method thread
step rn 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_eager 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-graph
step rn2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_eager2 300 python bench.py --model resnet50 --steps 20 --warmup 5 --no-graph
exit 0
