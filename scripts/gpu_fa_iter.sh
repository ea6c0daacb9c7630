#!/bin/bash
# FA iteration: numerics (flash tests) then per-kernel times at the GPT shape.
OUT=gpurun_out/${1:-fa_iter}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -k "flash or attention" -x -q --timeout 120 --timeout-method thread > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/k -o k --output-format csv -- python3 -m scripts.fa_one 16 16 1024 128 1 10 > $OUT/k.log 2>&1 || { tail -5 $OUT/k.log; exit 1; }
grep -E "^(fwd|bwd):" $OUT/k.log
python3 - "$OUT/k/k_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'fa::' in r['Name'] or 'attn_delta' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us  {r['Name'][:60]}")
PY
