#!/bin/bash
# Round 6 batch V: non-temporal epilogue store policies (PRA_PTS_NT 0/1/3/4/5) on the GPT bench.
OUT=gpurun_out/${1:-r6v}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6 | cut -c1-160; if fatal $rc; then exit $rc; fi; }
step nt5 200 env PRA_PTS_NT=5 python scripts/r6_dyn_probe.py
step nt3 200 env PRA_PTS_NT=3 python scripts/r6_dyn_probe.py
step b0 300 env PRA_PTS_NT=0 python bench.py --steps 20 --warmup 5
step b3 300 env PRA_PTS_NT=3 python bench.py --steps 20 --warmup 5
step b4 300 env PRA_PTS_NT=4 python bench.py --steps 20 --warmup 5
step b5 300 env PRA_PTS_NT=5 python bench.py --steps 20 --warmup 5
step b1 300 env PRA_PTS_NT=1 python bench.py --steps 20 --warmup 5
step b0b 300 env PRA_PTS_NT=0 python bench.py --steps 20 --warmup 5
step b3b 300 env PRA_PTS_NT=3 python bench.py --steps 20 --warmup 5
step b4b 300 env PRA_PTS_NT=4 python bench.py --steps 20 --warmup 5
step b5b 300 env PRA_PTS_NT=5 python bench.py --steps 20 --warmup 5
exit 0
