set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1 ; echo BENCH_EXIT $?
tail -3 gpurun_out/bench_gpt.log
