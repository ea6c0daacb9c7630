#!/bin/bash
# optimizer / next-forward overlap: GPU tests, then GPT A/B back to back, then a trace
OUT=gpurun_out/${1:-r3s}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_opt_overlap_gpu.py tests/test_rccl_gpu.py -x -v --timeout 120 --timeout-method thread
step gpt_on 300 python bench.py --gpus 1 --steps 20 --warmup 5
PRA_OPT_OVERLAP=0 step gpt_off 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_on2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gptprof 400 rocprofv3 --kernel-trace --stats -d $OUT/gptprof -o gpt --output-format csv -- python3 bench.py --gpus 1 --steps 4 --warmup 2
exit 0
