#!/bin/bash
# Round 6 batch T: per-XCD self-resetting tickets (no exit count / fence): GEMM tier, dyn A/B alone
# and under co-resident load, GPT bench.
OUT=gpurun_out/${1:-r6t}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step gemmtests 600 python -u -m pytest tests/test_gemm_lds_gpu.py tests/test_gemm_gpu.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider
step dyn1 200 env PRA_PTS_DYN=1 python scripts/r6_sp_probe.py
step dyn0 200 env PRA_PTS_DYN=0 python scripts/r6_sp_probe.py
step dyn1b 200 env PRA_PTS_DYN=1 python scripts/r6_sp_probe.py
step coload1 200 env PRA_PTS_DYN=1 python scripts/r6_dyn_probe.py
step coload0 200 env PRA_PTS_DYN=0 python scripts/r6_dyn_probe.py
step bench1 300 env PRA_PTS_DYN=1 python bench.py --steps 20 --warmup 5
step bench0 300 env PRA_PTS_DYN=0 python bench.py --steps 20 --warmup 5
exit 0
