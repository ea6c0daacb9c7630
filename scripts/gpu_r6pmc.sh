#!/bin/bash
# Round 6: PMC of the fused-epilogue fc1 GEMM vs the plain one (VALU vs MFMA work per dispatch).
OUT=gpurun_out/${1:-r6pmc}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 -s KILL "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; if fatal $rc; then exit $rc; fi; }
step pass1 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o p -- python scripts/r6_epi_pmc_probe.py
cp /tmp/pmc1/p_counter_collection.csv $OUT/pass1.csv
step pass2 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA TCC_EA0_WRREQ_sum --output-format csv -d /tmp/pmc2 -o p -- python scripts/r6_epi_pmc_probe.py
cp /tmp/pmc2/p_counter_collection.csv $OUT/pass2.csv
exit 0
