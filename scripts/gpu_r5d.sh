#!/bin/bash
# Round 5: PTS dy·Wᵀ epilogue cost breakdown (fc2 dgrad GPT and BERT shapes).
OUT=gpurun_out/${1:-r5d}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 12; if fatal $rc; then exit $rc; fi; }
step gpt 200 python scripts/gemm_epi_probe.py
step bert 200 python scripts/gemm_epi_probe.py 16384 3072 768
exit 0
