#!/bin/bash
# Round 6 batch Y: dK/dV query-split (QS) vs 4-wave kernel, causal and not, S 1024 / 2048.
OUT=gpurun_out/${1:-r6y}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "^[WE]2026" | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
for cfg in "1 1024 16" "0 1024 16" "1 2048 8" "0 2048 8"; do
  set -- $cfg
  for qs in 1 0; do
    step p_c$1_s$2_qs$qs 200 env PRA_FA_DKDV_QS=$qs rocprofv3 --kernel-trace --stats -d $OUT/p_c$1_s$2_qs$qs -o p -- python scripts/fa_probe.py --causal $1 --S $2 --B $3 --check 0
  done
done
exit 0
