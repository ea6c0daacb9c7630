#!/bin/bash
# FA backward dS path: numerics tests, both dQ paths timed, rocprof kernel stats of one fwd+bwd shape.
OUT=gpurun_out/${1:-fads}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_kernels_gpu.py -k flash -x -q --timeout 120 --timeout-method thread
step fa_ds 120 python -m scripts.fa_one 16 16 1024 128 1 50
step fa_sweep 120 env PRA_FA_DQ=sweep python -m scripts.fa_one 16 16 1024 128 1 50
step prof 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o fa --output-format csv -- python3 -m scripts.fa_one 16 16 1024 128 1 20
step bench 300 python bench.py --steps 20 --warmup 5
exit 0
