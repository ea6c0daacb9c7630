set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o gpt --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/prof_bench.log 2>&1; echo PROF_EXIT $?
find gpurun_out/prof -name "*stats*" | head
