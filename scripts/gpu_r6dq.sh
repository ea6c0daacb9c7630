#!/bin/bash
# Round 6: dQ (dS^T) kernel launch shapes on the causal GPT attention shape (PRA_FA_DQ_SHAPE; the old name PRA_FA_DQ also switched the Python dQ path to the sweep kernel).
OUT=gpurun_out/${1:-r6dq}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; if fatal $rc; then exit $rc; fi; }
for v in 8x3 8x2 4x3 4x4; do
  step dq_$v 200 env PRA_FA_DQ_SHAPE=$v rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/dq_$v -o p -- python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 1
  cp /tmp/dq_$v/p_kernel_stats.csv $OUT/dq_${v}_stats.csv
done
exit 0
