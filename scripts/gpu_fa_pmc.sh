#!/bin/bash
# Flash-attention timing + counter passes (kernel-trace only, one pmc set per run).
OUT=gpurun_out/${1:-fa_pmc}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 python3 -m scripts.fa_one 16 16 1024 128 1 20 > $OUT/time.log 2>&1 || { tail -5 $OUT/time.log; exit 1; }
cat $OUT/time.log
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $OUT/p$i -o p --output-format csv -- python3 -m scripts.fa_one 16 16 1024 128 1 3 > $OUT/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo ok
