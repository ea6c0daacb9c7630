#!/bin/bash
# BERT with the caching allocator vs the native allocator: bench + kernel traces of both
OUT=gpurun_out/${1:-r3t}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step bert_torch 300 python bench.py --model bert-base --steps 20 --warmup 5
PRA_ALLOCATOR=auto_growth step bert_native 300 python bench.py --model bert-base --steps 20 --warmup 5
step prof_torch 300 rocprofv3 --kernel-trace -d $OUT/pt -o bt --output-format csv -- python3 bench.py --model bert-base --steps 6 --warmup 3
PRA_ALLOCATOR=auto_growth step prof_native 300 rocprofv3 --kernel-trace -d $OUT/pn -o bn --output-format csv -- python3 bench.py --model bert-base --steps 6 --warmup 3
exit 0
