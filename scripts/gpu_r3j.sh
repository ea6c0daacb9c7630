#!/bin/bash
# ResNet 1x1 stats A/B (shape-gated) and GPT fc2-dgrad dGELU epilogue A/B.
OUT=gpurun_out/${1:-r3j}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 400 python -u -m pytest tests/test_conv_bn_stats_gpu.py tests/test_resnet_unit.py -m gpu -q -x --timeout 120 --timeout-method thread
step rn_new 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_old 300 env PRA_CONV1X1_STATS=0 python bench.py --model resnet50 --steps 20 --warmup 5
step gpt_epi 300 env PRA_MLP_DGELU_EPI=1 python bench.py --steps 10 --warmup 3
step gpt_base 300 python bench.py --steps 10 --warmup 3
step rn_new2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_old2 300 env PRA_CONV1X1_STATS=0 python bench.py --model resnet50 --steps 20 --warmup 5
step gpt_epi2 300 env PRA_MLP_DGELU_EPI=1 python bench.py --steps 10 --warmup 3
step gpt_base2 300 python bench.py --steps 10 --warmup 3
exit 0
