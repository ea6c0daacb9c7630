#!/bin/bash
# Round 5: add+dropout+LN backward with the row stashed in LDS between its two passes (A/B).
OUT=gpurun_out/${1:-r5aj}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_grad_accum_gpu.py tests/test_tp_fused.py -k "adl or dropout or layer_norm or ln or add" -m gpu -x -q --timeout 120 --timeout-method thread
step gpt 300 python bench.py --steps 10 --warmup 3
PRA_ADL_NBLK=512 step gpt_512 300 python bench.py --steps 10 --warmup 3
PRA_ADL_STASH=0 step gpt_old 300 python bench.py --steps 10 --warmup 3
step gpt2 300 python bench.py --steps 10 --warmup 3
PRA_ADL_NBLK=512 step gpt_512b 300 python bench.py --steps 10 --warmup 3
PRA_ADL_STASH=0 step gpt_old2 300 python bench.py --steps 10 --warmup 3
step bert 300 python bench.py --model bert --steps 20 --warmup 5
PRA_ADL_STASH=0 step bert_old 300 python bench.py --model bert --steps 20 --warmup 5
exit 0
