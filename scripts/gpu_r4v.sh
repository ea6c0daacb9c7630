#!/bin/bash
# fc2 dgrad through the gemm() shape policy (short K -> in-tree persistent kernel): BERT A/B.
OUT=gpurun_out/${1:-r4v}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log) $(grep -v amdgpu.ids $OUT/$name.log | tail -n 1 | cut -c1-120)"; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemm_lds_gpu.py -k "mlp or auto_policy" tests/test_bert_gpu.py
for i in 1 2; do
  step on_$i 300 python bench.py --model bert-base --steps 40 --warmup 5
  step off_$i 300 env PRA_GEMM_NT_SHORTK=0 python bench.py --model bert-base --steps 40 --warmup 5
done
exit 0
