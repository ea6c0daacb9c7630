#!/bin/bash
# TunableOp tuning of the BERT step's library GEMMs (op-by-op executor: no graph capture while
# tuning), merged with the GPT solutions, then a BERT A/B.
OUT=gpurun_out/${1:-r4ag}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -o '"ms_per_step": [0-9.]*' $OUT/$name.log)"; if fatal $rc; then exit $rc; fi; }
step tune 900 env PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=30 \
  PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=200 PYTORCH_TUNABLEOP_FILENAME=$OUT/bert_tune.csv \
  python -u bench.py --model bert-base --steps 2 --warmup 1 --no-graph --no-tuned-gemms
ls $OUT
exit 0
