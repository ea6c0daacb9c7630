#!/bin/bash
OUT=gpurun_out/${1:-r5ah}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_flash_ext.py -k other_head_dims -m gpu -x -q -s --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1; echo "rc=$?"; grep -E "peak|passed|failed|Error" $OUT/tests.log | head -20
