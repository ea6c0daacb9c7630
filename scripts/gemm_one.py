"""Run one GEMM shape repeatedly (ours or hipBLASLt) for rocprofv3 counter passes.
    python scripts/gemm_one.py {ours|blas} layout M N K [iters]"""
import sys
import torch
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from scripts.gemm_lds_bench import operands, ref_mm, ours  # noqa: E402

which, layout, M, N, K = sys.argv[1], *map(int, sys.argv[2:6])
it = int(sys.argv[6]) if len(sys.argv) > 6 else 10
a, b = operands(layout, M, N, K, torch.device('cuda'))
c = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
for _ in range(it):
    if which == 'ours':
        ours(layout, a, b, c, M, N, K)
    else:
        ref_mm(layout, a, b)
torch.cuda.synchronize()
print('done', flush=True)
