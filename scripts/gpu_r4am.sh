#!/bin/bash
# Same-box A/B of two builds of the extension (abtmp/base.so vs abtmp/fwd4.so): FA probes, tests, BERT step.
OUT=gpurun_out/${1:-r4am}
mkdir -p $OUT
export TMPDIR=/tmp PRA_SKIP_PROVENANCE=1
SO=paddle_ray_amd/ops/_pra_hip.cpython-310-x86_64-linux-gnu.so
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc] $(grep -v amdgpu.ids $OUT/$name.log | grep -E 'fwd4out|ms_per_step' | tr '\n' ' ' | cut -c1-260)"; if fatal $rc; then exit $rc; fi; }
for i in 1 2; do
  for v in base fwd4; do
    cp abtmp/$v.so $SO
    true
    step ${v}_bert_$i 120 python scripts/fa_ext_probe.py --iters 30
  done
done
cp abtmp/fwd4.so $SO
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_flash_ext.py tests/test_kernels_gpu.py tests/test_bert_gpu.py tests/test_static.py
for v in base fwd4; do
  cp abtmp/$v.so $SO
  step ${v}_bert 300 python bench.py --model bert-base --steps 40 --warmup 5
  step ${v}_bertb 300 python bench.py --model bert-base --steps 40 --warmup 5
done
cp abtmp/fwd4.so $SO
exit 0
