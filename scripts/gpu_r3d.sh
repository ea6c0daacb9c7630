#!/bin/bash
# GEMM configuration A/B (W8 / W4 / W8I / hipBLASLt) + numerics, wave-state counters on dy·Wᵀ,
# ResNet50 and GPT step profiles.
OUT=gpurun_out/${1:-r3d}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; tail -n 6 $OUT/$name.log; if fatal $rc; then exit $rc; fi; }
step gemmtest 300 python -u -m pytest tests/test_gemm_lds_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread
step gemmab 300 python scripts/gemm_lds_bench.py --w4
step pmc 600 bash scripts/gpu_gemm_pmc3.sh r3d/pmc
step resnet 300 python bench.py --model resnet50 --steps 10 --warmup 3
step rnprof 300 rocprofv3 --kernel-trace --stats -d $OUT/rnprof -o rn --output-format csv -- python3 bench.py --model resnet50 --steps 3 --warmup 2
step gptprof 300 rocprofv3 --kernel-trace --stats -d $OUT/gptprof -o gpt --output-format csv -- python3 bench.py --steps 5 --warmup 2
exit 0
