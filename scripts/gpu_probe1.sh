#!/bin/bash
# Probe run: GEMM library/layout table + flash-attention timing and PMC counters.
mkdir -p gpurun_out/probe1
cd /root/repo
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; echo "[rc=$rc] $*"; if fatal $rc; then exit $rc; fi; return 0; }
run 200 python scripts/fa_probe.py > gpurun_out/probe1/fa.log 2>&1
cat gpurun_out/probe1/fa.log
run 200 rocprofv3 --kernel-trace --stats -d gpurun_out/probe1/fa_trace -o fa --output-format csv -- python3 scripts/fa_probe.py --check 0 --iters 5 > gpurun_out/probe1/fa_trace.log 2>&1
run 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS -d gpurun_out/probe1/pmc1 -o pmc1 --output-format csv -- python3 scripts/fa_probe.py --check 0 --iters 2 > gpurun_out/probe1/pmc1.log 2>&1
run 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/probe1/pmc2 -o pmc2 --output-format csv -- python3 scripts/fa_probe.py --check 0 --iters 2 > gpurun_out/probe1/pmc2.log 2>&1
run 300 python scripts/gemm_probe.py --lib hipblaslt > gpurun_out/probe1/gemm_hipblaslt.log 2>&1
run 300 python scripts/gemm_probe.py --lib rocblas > gpurun_out/probe1/gemm_rocblas.log 2>&1
run 600 python scripts/gemm_probe.py --lib hipblaslt --tunable > gpurun_out/probe1/gemm_tunable.log 2>&1
tail -n 32 gpurun_out/probe1/gemm_*.log
