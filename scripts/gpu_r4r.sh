#!/bin/bash
# QKV bias gradient from the flash backward's column-sum partials: tests, then GPT / BERT A/B.
OUT=gpurun_out/${1:-r4r}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 2 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_flash_ext.py tests/test_bert_gpu.py tests/test_static.py
step gpt_on 300 python bench.py --steps 12 --warmup 4
step gpt_off 300 env PRA_FA_BIAS_PART=0 python bench.py --steps 12 --warmup 4
step bert_on 300 python bench.py --model bert-base --steps 30 --warmup 5
step bert_off 300 env PRA_FA_BIAS_PART=0 python bench.py --model bert-base --steps 30 --warmup 5
step gpt_on2 300 python bench.py --steps 12 --warmup 4
step gpt_off2 300 env PRA_FA_BIAS_PART=0 python bench.py --steps 12 --warmup 4
exit 0
