#!/bin/bash
# Round 6 batch S: where the dynamic-order ticket is consumed (after step 0 vs after the steady loop).
OUT=gpurun_out/${1:-r6s}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step late_t 300 env PRA_PTS_VAR=1048576 python -u -m pytest tests/test_gemm_lds_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "many_tiles or layouts"
step dyn1 200 env PRA_PTS_DYN=1 python scripts/r6_sp_probe.py
step late 200 env PRA_PTS_DYN=1 PRA_PTS_VAR=1048576 python scripts/r6_sp_probe.py
step dyn0 200 env PRA_PTS_DYN=0 python scripts/r6_sp_probe.py
step late2 200 env PRA_PTS_DYN=1 PRA_PTS_VAR=1048576 python scripts/r6_sp_probe.py
step dyn0v 200 env PRA_PTS_DYN=0 PRA_PTS_VAR=1048576 python scripts/r6_sp_probe.py
exit 0
