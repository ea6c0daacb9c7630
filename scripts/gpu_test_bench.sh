set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kernels.log 2>&1; echo TEST_EXIT $?
tail -5 gpurun_out/kernels.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_gpt.log 2>&1 ; echo BENCH_EXIT $?
tail -1 gpurun_out/bench_gpt.log
