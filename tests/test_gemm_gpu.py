"""MFMA GEMM + bias + activation kernel (ops/csrc/gemm.hip) vs a PyTorch fp32 reference
(parity: reference fused_gemm_epilogue / fused_matmul_bias tests,
python/paddle/fluid/tests/unittests/test_fused_matmul_bias.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from paddle_ray_amd.ops import fused as F  # noqa: E402
from paddle_ray_amd.ops import registry as R  # noqa: E402
from paddle_ray_amd.ops import _native  # noqa: E402


def _ref(x, w, b, act):
    z = x.float() @ w.float() + (b.float() if b is not None else 0)
    return F._act_ref(z, F._ACT[act])


@pytest.mark.parametrize('dtype', [torch.bfloat16, torch.float16])
@pytest.mark.parametrize('shape', [(256, 512, 384), (77, 200, 136), (1, 8, 8), (1000, 1024, 2048),
                                   (130, 72, 4104), (12296, 4104, 136),
                                   (8192, 4096, 4096)])
@pytest.mark.parametrize('act', [None, 'gelu', 'gelu_tanh', 'relu'])
def test_gemm_bias_act_fwd(dtype, shape, act):
    _native.require()
    M, N, K = shape
    torch.manual_seed(0)
    x = torch.randn(M, K, device='cuda', dtype=dtype)
    w = torch.randn(K, N, device='cuda', dtype=dtype) / K ** 0.5
    b = torch.randn(N, device='cuda', dtype=dtype)
    R.reset_stats()
    y = F.gemm_bias_act(x, w, b, act)
    torch.cuda.synchronize()
    assert R.stats().get(('gemm_bias_act', 'hip'), 0) == 1
    ref = _ref(x, w, b, act)
    tol = 2e-2 if dtype == torch.bfloat16 else 4e-3
    torch.testing.assert_close(y.float(), ref, atol=tol, rtol=tol)


def test_gemm_strided_and_nobias():
    _native.require()
    torch.manual_seed(1)
    big = torch.randn(300, 640, device='cuda', dtype=torch.bfloat16)
    x = big[:, :512]  # lda = 640
    w = torch.randn(512, 264, device='cuda', dtype=torch.bfloat16) / 512 ** 0.5
    y = F.GemmBiasActFn.apply(x, w, None, 0)
    torch.testing.assert_close(y.float(), x.float() @ w.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize('act', [None, 'gelu', 'relu'])
def test_gemm_bias_act_backward(act):
    _native.require()
    torch.manual_seed(2)
    x = torch.randn(4, 96, 256, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(256, 512, device='cuda', dtype=torch.bfloat16) / 16).requires_grad_(True)
    b = torch.randn(512, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    y = F.gemm_bias_act(x, w, b, act)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    F._act_ref(xr @ wr + br, F._ACT[act]).backward(g.float())
    for a, r in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        scale = r.abs().max().item() + 1e-6
        assert (a.float() - r).abs().max().item() / scale < 3e-2


def test_fused_linear_activation_runs_mfma():
    import paddle_ray_amd as paddle
    from paddle_ray_amd.incubate.nn import functional as IF
    _native.require()
    x = torch.randn(64, 256, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(512, 256, device='cuda', dtype=torch.bfloat16) / 16
    b = torch.randn(512, device='cuda', dtype=torch.bfloat16)
    R.reset_stats()
    y = IF.fused_linear_activation(paddle.Tensor(x), paddle.Tensor(w), paddle.Tensor(b), trans_y=True,
                                   activation='gelu')
    assert R.stats().get(('gemm_bias_act', 'hip'), 0) == 1
    ref = torch.nn.functional.gelu(x.float() @ w.float().t() + b.float())
    torch.testing.assert_close(y._t.float(), ref, atol=2e-2, rtol=2e-2)
