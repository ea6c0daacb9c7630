#!/bin/bash
# Round 6 batch X: flash attention fwd/bwd, causal vs non-causal at S 1024 / 2048 (per-kernel stats).
OUT=gpurun_out/${1:-r6x}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "^[WE]2026" | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step c1024 120 python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 0
step n1024 120 python scripts/fa_probe.py --causal 0 --S 1024 --B 16 --check 0
step c2048 120 python scripts/fa_probe.py --causal 1 --S 2048 --B 8 --check 0
step n2048 120 python scripts/fa_probe.py --causal 0 --S 2048 --B 8 --check 0
step c4096 120 python scripts/fa_probe.py --causal 1 --S 4096 --B 4 --check 0
step pc1024 200 rocprofv3 --kernel-trace --stats -d $OUT/pc1024 -o p -- python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 0
step pn1024 200 rocprofv3 --kernel-trace --stats -d $OUT/pn1024 -o p -- python scripts/fa_probe.py --causal 0 --S 1024 --B 16 --check 0
exit 0
