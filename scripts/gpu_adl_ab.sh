#!/bin/bash
# add+dropout+LN backward: two-pass (default) vs one-pass (PRA_ADL_BWD=1), numerics + GPT A/B + kernel time.
OUT=gpurun_out/${1:-adl_ab}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 2 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_accum_gpu.py tests/test_tp_fused.py -m gpu -x -q --timeout 120 --timeout-method thread
step two_a 200 python bench.py --steps 20 --warmup 5
step one_a 200 env PRA_ADL_BWD=1 python bench.py --steps 20 --warmup 5
step two_b 200 python bench.py --steps 20 --warmup 5
step one_b 200 env PRA_ADL_BWD=1 python bench.py --steps 20 --warmup 5
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
exit 0
