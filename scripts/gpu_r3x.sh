#!/bin/bash
# narrow (Cout <= 128) conv weight gradient on 128-row tiles (128-wide M-contiguous dy image):
# full GPU suite, per-shape table, ResNet A/B, then GPT to confirm the GEMM paths are unchanged
OUT=gpurun_out/${1:-r3x}
mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 1 $OUT/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step conv 300 python -u -m pytest tests/test_conv_kxk.py -x -q --timeout 120 --timeout-method thread
step tests 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
step wgrad 200 python scripts/conv_wgrad_bench.py
step rn_on 300 python bench.py --model resnet50 --steps 20 --warmup 5
PRA_CONV_WGRAD_NARROW=0 step rn_off 300 python bench.py --model resnet50 --steps 20 --warmup 5
step rn_on2 300 python bench.py --model resnet50 --steps 20 --warmup 5
step gpt 300 python bench.py --gpus 1 --steps 20 --warmup 5
exit 0
