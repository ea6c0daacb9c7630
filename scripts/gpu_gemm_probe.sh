#!/bin/bash
# GEMM probe: hipBLASLt vs rocBLAS vs TunableOp on the GPT-3 1.3B GEMM shapes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_probe.py --lib hipblaslt > gpurun_out/gemm_hipblaslt.log 2>&1 &&
timeout -k 10 300 python scripts/gemm_probe.py --lib rocblas > gpurun_out/gemm_rocblas.log 2>&1 &&
timeout -k 10 600 python scripts/gemm_probe.py --lib hipblaslt --tunable > gpurun_out/gemm_tunable.log 2>&1
rc=$?
tail -n 40 gpurun_out/gemm_*.log
exit $rc
