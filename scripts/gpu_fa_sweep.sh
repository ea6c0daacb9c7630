#!/bin/bash
OUT=gpurun_out/${1:-fasweep}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in "--causal 1" "--causal 0" "--causal 1 --S 2048 --B 8" "--causal 0 --S 2048 --B 8" "--causal 0 --D 64 --H 32" "--causal 1 --S 4096 --B 4"; do
  timeout -k 10 120 python scripts/fa_probe.py $cfg --check 0 >> $OUT/sweep.log 2>&1 || exit $?
  echo "  ^ $cfg" >> $OUT/sweep.log
done
grep -v amdgpu.ids $OUT/sweep.log
