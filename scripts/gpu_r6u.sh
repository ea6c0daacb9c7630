#!/bin/bash
# Round 6 batch U: non-temporal epilogue stores in the persistent GEMM (PRA_PTS_NT) A/B.
OUT=gpurun_out/${1:-r6u}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step nt_t 300 env PRA_PTS_NT=1 python -u -m pytest tests/test_gemm_lds_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "many_tiles or epilogue or mulz"
step ep0 200 env PRA_PTS_NT=0 python scripts/r6_dyn_probe.py
step ep1 200 env PRA_PTS_NT=1 python scripts/r6_dyn_probe.py
step sp1 200 env PRA_PTS_NT=1 python scripts/r6_sp_probe.py
step sp0 200 env PRA_PTS_NT=0 python scripts/r6_sp_probe.py
step ep1b 200 env PRA_PTS_NT=1 python scripts/r6_dyn_probe.py
step ep0b 200 env PRA_PTS_NT=0 python scripts/r6_dyn_probe.py
step bench1 300 env PRA_PTS_NT=1 python bench.py --steps 20 --warmup 5
step bench0 300 env PRA_PTS_NT=0 python bench.py --steps 20 --warmup 5
exit 0
