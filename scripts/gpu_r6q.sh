#!/bin/bash
# Round 6 batch Q: GEMM tier (self-resetting counters, capture-safe counter pool), K-stagger sweep.
OUT=gpurun_out/${1:-r6q}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step gemmtests 600 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step gemmtests_stg 600 env PRA_PTS_STG=3 python -u -m pytest tests/test_gemm_lds_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "many_tiles or layouts or mulz or gelu_derivative"
step stg0 200 env PRA_PTS_STG=0 python scripts/r6_sp_probe.py
step stg1 200 env PRA_PTS_STG=1 python scripts/r6_sp_probe.py
step stg2 200 env PRA_PTS_STG=2 python scripts/r6_sp_probe.py
step stg4 200 env PRA_PTS_STG=4 python scripts/r6_sp_probe.py
step stg8 200 env PRA_PTS_STG=8 python scripts/r6_sp_probe.py
step stg0b 200 env PRA_PTS_STG=0 python scripts/r6_sp_probe.py
exit 0
