#!/bin/bash
# Round 5: LM-head weight gradient with the 40-tile tail split off (GPT A/B).
OUT=gpurun_out/${1:-r5ad}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_gemm_lds_gpu.py -k "tail or paired" -m gpu -x -q --timeout 120 --timeout-method thread
step gpt 300 python bench.py --steps 10 --warmup 3
PRA_GEMM_TN_TAIL=0 step gpt_old 300 python bench.py --steps 10 --warmup 3
step gpt2 300 python bench.py --steps 10 --warmup 3
PRA_GEMM_TN_TAIL=0 step gpt_old2 300 python bench.py --steps 10 --warmup 3
PRA_ADL_NBLK=512 step gpt_nb512 300 python bench.py --steps 10 --warmup 3
PRA_ADL_NBLK=1536 step gpt_nb1536 300 python bench.py --steps 10 --warmup 3
exit 0
