#!/bin/bash
# TS default: MHA dropout test, GPT A/B (dGELU epilogue), BERT, GPT + BERT rocprofv3 kernel stats.
OUT=gpurun_out/${1:-r4j}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3; if fatal $rc; then exit $rc; fi; }
step fatests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_flash_ext.py
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_dgelu 300 env PRA_MLP_DGELU_EPI=1 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt2 300 python bench.py --gpus 1 --steps 20 --warmup 5
step gpt_dgelu2 300 env PRA_MLP_DGELU_EPI=1 python bench.py --gpus 1 --steps 20 --warmup 5
step bert 300 python bench.py --model bert-base --steps 20 --warmup 5
step resnet 300 python bench.py --model resnet50 --steps 20 --warmup 5
step profgpt 300 rocprofv3 --kernel-trace --stats -d $OUT/profgpt -o gpt --output-format csv -- python3 bench.py --steps 2 --warmup 1
step profbert 300 rocprofv3 --kernel-trace --stats -d $OUT/profbert -o bert --output-format csv -- python3 bench.py --model bert-base --steps 2 --warmup 1
exit 0
