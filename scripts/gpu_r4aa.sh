#!/bin/bash
OUT=gpurun_out/${1:-r4aa}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 6; if fatal $rc; then exit $rc; fi; }
step gpt 120 python scripts/fa_probe.py --iters 30
step gpt2 120 python -m scripts.fa_one 16 16 1024 128 1 20
step bert 120 python scripts/fa_ext_probe.py --iters 30
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_flash_ext.py tests/test_kernels_gpu.py -k "flash or fa_ or attention or qkv"
exit 0
