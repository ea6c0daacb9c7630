#!/bin/bash
# Round 6 batch F: GPU tests of the round's new paths; profiler correlation probe.
OUT=gpurun_out/${1:-r6f}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 14 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step passes 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_distributed_passes.py tests/test_dist_fused_lamb.py -m gpu

step proftest 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_profiler_gpu.py -m gpu
exit 0
