#!/bin/bash
# Tune GPT GEMMs with TunableOp, then A/B the bench with / without the tuned solutions.
OUT=gpurun_out/${1:-tune}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tune 1000 python -u scripts/tune_gemms.py --out $OUT/gemm_gfx950.csv --steps 2
export PRA_GEMM_TUNING_FILE=$OUT/gemm_gfx950.csv
step tuned 300 python bench.py --steps 20 --warmup 5
step untuned 300 python bench.py --steps 20 --warmup 5 --no-tuned-gemms
exit 0
