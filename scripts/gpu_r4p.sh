#!/bin/bash
# dQ = dS K launch-shape A/B (PRA_FA_DQ): GPT and BERT attention shapes, with numerics checks.
OUT=gpurun_out/${1:-r4p}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6; if fatal $rc; then exit $rc; fi; }
for v in 8x3 8x2 4x3 4x4; do
  step gpt_$v 120 env PRA_FA_DQ=$v python scripts/fa_probe.py --iters 30
  step bert_$v 120 env PRA_FA_DQ=$v python scripts/fa_ext_probe.py --iters 30
done
exit 0
