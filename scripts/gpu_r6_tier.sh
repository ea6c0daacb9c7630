#!/bin/bash
# GPU tier + smoke on the current tree.
OUT=gpurun_out/${1:-r6_tier}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 124|137|134|139) return 0;; esac; return 1; }
step() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1; local rc=$?;
         echo "[$name rc=$rc]"; grep -v amdgpu.ids $OUT/$name.log | tail -n 3 | cut -c1-250; if fatal $rc; then exit $rc; fi; }
step tests 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider
step smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python bench.py --steps 20 --warmup 5
exit 0
