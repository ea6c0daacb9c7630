#!/bin/bash
# Round 5: BN-dgrad fusion probe after the epilogue Z/keep-bit prefetch.
OUT=gpurun_out/${1:-r5q}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-200; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_bn_dgrad_fuse.py -x -q --timeout 120 --timeout-method thread
step probe 300 python scripts/bn_dgrad_probe.py
exit 0
