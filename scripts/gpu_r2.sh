#!/bin/bash
# Round-2 GPU check: GPU tests, the driver's exact bench line, rocprofv3 kernel stats.
# Stops at the first failing / faulting / timed-out step.
OUT=gpurun_out/${1:-r2}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 3 $OUT/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
step prof 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o gpt --output-format csv -- python3 bench.py --steps 3 --warmup 2
exit 0
