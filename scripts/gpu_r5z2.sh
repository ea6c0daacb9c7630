#!/bin/bash
OUT=gpurun_out/${1:-r5z2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/graph_capture_probe.py 16 > $OUT/probe.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids $OUT/probe.log | grep -v "^  warn" | tail -40
