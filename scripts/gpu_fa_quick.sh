#!/bin/bash
# Quick flash-attention timing + numerics check + kernel trace.
mkdir -p gpurun_out/faq
export TMPDIR=/tmp
timeout -k 10 300 python scripts/fa_probe.py > gpurun_out/faq/fa.log 2>&1 && cat gpurun_out/faq/fa.log &&
timeout -k 10 300 python scripts/fa_probe.py --causal 0 --check 0 >> gpurun_out/faq/fa.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/faq/trace -o fa --output-format csv -- python3 scripts/fa_probe.py --check 0 --iters 5 > gpurun_out/faq/trace.log 2>&1
rc=$?
cat gpurun_out/faq/fa.log
exit $rc
