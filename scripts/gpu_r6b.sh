#!/bin/bash
# Round 6 batch B: new GPU tests (Lamb shard kernels, profiler device side), PMC of the in-tree
# persistent dy·Wᵀ kernel vs hipBLASLt at fc1.dgrad, GPT step kernel table.
OUT=gpurun_out/${1:-r6b}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 8 | cut -c1-220; if fatal $rc; then exit $rc; fi; }
step tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dist_fused_lamb.py tests/test_profiler_gpu.py tests/test_distributed_passes.py -m gpu
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_MFMA,SQ_WAIT_INST_LDS,GRBM_GUI_ACTIVE
P2=SQ_INSTS_LDS,SQ_INSTS_VMEM,SQ_INSTS_SALU,SQ_INSTS_VALU,SQ_LDS_BANK_CONFLICT,SQ_INSTS_SMEM,SQ_LDS_IDX_ACTIVE,SQ_INSTS_BRANCH
P3=TCC_HIT_sum,TCC_MISS_sum,TCC_EA0_RDREQ_sum
for who in ours blas; do
  for p in 1 2 3; do
    eval C=\$P$p
    PRA_GEMM_PTS=2 step pmc_${who}_$p 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$who -o p$p -- python scripts/gemm_one.py $who 1 16384 2048 8192 4
  done
done
step gpt_prof 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/gpt_prof -o gpt -- python bench.py --steps 4 --warmup 3
python scripts/trace_window.py $OUT/gpt_prof/gpt_kernel_trace.csv adamw_mt 3 45 > $OUT/gpt_table.md 2>&1; head -30 $OUT/gpt_table.md
exit 0
