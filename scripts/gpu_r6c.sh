#!/bin/bash
# Round 6 batch C: refill spacing of the persistent W4 GEMM; new GPU tests (lamb, passes, profiler).
OUT=gpurun_out/${1:-r6c}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 12 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
for sp in 0 2 3; do
  PRA_PTS_SP=$sp step sp$sp 240 python scripts/r6_sp_probe.py
done
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dist_fused_lamb.py tests/test_profiler_gpu.py tests/test_distributed_passes.py -m gpu
exit 0
