#!/bin/bash
OUT=gpurun_out/${1:-r5ae}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/strided_dgrad_bn_probe.py > $OUT/probe.log 2>&1; echo "rc=$?"; grep "|" $OUT/probe.log; tail -3 $OUT/probe.log
