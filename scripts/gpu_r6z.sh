#!/bin/bash
# Round 6 batch Z: persistent dK/dV (PRA_FA_DKDV_PERSIST): GPU tier, flash probe A/B, GPT bench A/B.
OUT=gpurun_out/${1:-r6z}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | grep -v "^[WE]2026" | tail -n 3 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step fa_check 120 python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 1
step fatests 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -k "flash or attn or attention or fa_"
step p1 200 env PRA_FA_DKDV_PERSIST=1 rocprofv3 --kernel-trace --stats -d $OUT/p1 -o p -- python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 0
step p0 200 env PRA_FA_DKDV_PERSIST=0 rocprofv3 --kernel-trace --stats -d $OUT/p0 -o p -- python scripts/fa_probe.py --causal 1 --S 1024 --B 16 --check 0
step n1 200 env PRA_FA_DKDV_PERSIST=1 rocprofv3 --kernel-trace --stats -d $OUT/n1 -o p -- python scripts/fa_probe.py --causal 0 --S 1024 --B 16 --check 0
step n0 200 env PRA_FA_DKDV_PERSIST=0 rocprofv3 --kernel-trace --stats -d $OUT/n0 -o p -- python scripts/fa_probe.py --causal 0 --S 1024 --B 16 --check 0
step b1 300 env PRA_FA_DKDV_PERSIST=1 python bench.py --steps 20 --warmup 5
step b0 300 env PRA_FA_DKDV_PERSIST=0 python bench.py --steps 20 --warmup 5
step b1b 300 env PRA_FA_DKDV_PERSIST=1 python bench.py --steps 20 --warmup 5
step b0b 300 env PRA_FA_DKDV_PERSIST=0 python bench.py --steps 20 --warmup 5
exit 0
