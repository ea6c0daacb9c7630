#!/bin/bash
# FA probe timing + one PMC pass (8 SQ counters) on the GPT attention shape.
OUT=gpurun_out/${1:-fapmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python scripts/fa_probe.py --iters 20 > $OUT/probe.log 2>&1; rc=$?; cat $OUT/probe.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $OUT/pmc -o fa -- python3 scripts/fa_probe.py --iters 2 --check 0 > $OUT/pmc.log 2>&1; echo "pmc rc=$?"
exit 0
