#!/bin/bash
# Round 6 batch M: GEMM GPU tests with the compiler-tracked dynamic tile fetch; static vs dynamic.
OUT=gpurun_out/${1:-r6m}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step gemmtests 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gemm_lds_gpu.py tests/test_gemm_gpu.py -m gpu
PRA_PTS_DYN=0 step dyn0 180 python scripts/r6_dyn_probe.py
PRA_PTS_DYN=1 step dyn1 180 python scripts/r6_dyn_probe.py
PRA_PTS_DYN=0 step dyn0b 180 python scripts/r6_dyn_probe.py
PRA_PTS_DYN=1 step dyn1b 180 python scripts/r6_dyn_probe.py
exit 0
