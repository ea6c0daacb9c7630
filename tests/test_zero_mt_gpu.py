"""Multi-tensor zero fill (ops.fused.zero_tensors, the optimizer's clear_grad): one HIP launch
zeroes every tensor, including sizes that are not multiples of 16 bytes and > 64 KB pieces."""
import pytest
import torch

from paddle_ray_amd.ops import fused as K
from paddle_ray_amd.ops import _native


@pytest.mark.gpu
def test_zero_tensors_one_launch():
    assert _native.available()
    ts = [torch.randn(n, device='cuda').to(dt) for n, dt in
          ((1, torch.float32), (7, torch.bfloat16), (1000, torch.float32), (65536 * 3 + 5, torch.bfloat16),
           (4096, torch.float16), (262144, torch.float32))]
    guard = torch.randn(1024, device='cuda')
    g0 = guard.clone()
    K.zero_tensors(ts)
    K.zero_tensors(ts)  # cached plan
    torch.cuda.synchronize()
    assert all(int(torch.count_nonzero(t)) == 0 for t in ts)
    assert torch.equal(guard, g0)
