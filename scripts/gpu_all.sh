set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kernels.log 2>&1; echo TEST_EXIT $?
tail -3 gpurun_out/kernels.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1 ; echo BENCH_EXIT $?
tail -1 gpurun_out/bench_gpt.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o gpt --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_bench.log 2>&1; echo PROF_EXIT $?
