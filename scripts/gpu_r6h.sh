#!/bin/bash
# Round 6 batch H: AdamW two-group unroll A/B, optimizer kernel tests, profiler GPU test.
OUT=gpurun_out/${1:-r6h}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adam or Adam" tests/test_profiler_gpu.py -m gpu
PRA_ADAMW_X2=0 step ab0 120 python scripts/r6_adamw_ab.py
PRA_ADAMW_X2=1 step ab1 120 python scripts/r6_adamw_ab.py
PRA_ADAMW_X2=0 step ab0b 120 python scripts/r6_adamw_ab.py
PRA_ADAMW_X2=1 step ab1b 120 python scripts/r6_adamw_ab.py
exit 0
