#!/bin/bash
# Round 6 batch R: dynamic vs static persistent tile order on the plain GPT GEMM shapes (alone).
OUT=gpurun_out/${1:-r6r}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-300; if fatal $rc; then exit $rc; fi; }
step dyn1a 200 env PRA_PTS_DYN=1 python scripts/r6_sp_probe.py
step dyn0a 200 env PRA_PTS_DYN=0 python scripts/r6_sp_probe.py
step dyn1b 200 env PRA_PTS_DYN=1 python scripts/r6_sp_probe.py
step coload 200 python scripts/r6_dyn_probe.py
step dyn0b 200 env PRA_PTS_DYN=0 python scripts/r6_sp_probe.py
exit 0
