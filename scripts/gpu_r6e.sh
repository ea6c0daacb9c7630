#!/bin/bash
# Round 6 batch E: persistent W4 GEMM variants (MUBUF DMA, A-first fragment order, earlier
# second barrier) on the GPT shapes; GPU tests.
OUT=gpurun_out/${1:-r6e}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 12 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
PRA_PTS_BUF=0 PRA_PTS_VAR=0 step v0 240 python scripts/r6_sp_probe.py
PRA_PTS_BUF=1 PRA_PTS_VAR=0 step vb 240 python scripts/r6_sp_probe.py
PRA_PTS_BUF=0 PRA_PTS_VAR=256 step va 240 python scripts/r6_sp_probe.py
PRA_PTS_BUF=0 PRA_PTS_VAR=16640 step vab 240 python scripts/r6_sp_probe.py
PRA_PTS_BUF=0 PRA_PTS_VAR=16384 step vsh 240 python scripts/r6_sp_probe.py
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dist_fused_lamb.py tests/test_profiler_gpu.py tests/test_distributed_passes.py -m gpu
exit 0
