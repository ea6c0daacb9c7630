"""paddle.sparse products / elementwise / softmax / attention computed on coordinates
(sparse/ops.py) against dense fp64 references, including gradients w.r.t. values and dense
operands (parity targets: the reference's test_sparse_matmul_op.py, test_sparse_elementwise_op.py,
test_sparse_softmax_op.py, test_sparse_fused_attention_op.py)."""
import numpy as np
import pytest
import torch

import paddle_ray_amd as paddle
from paddle_ray_amd import sparse as SP
from paddle_ray_amd.sparse import nn as SN


def _rand_sparse(shape, density, seed, layout='coo'):
    g = torch.Generator().manual_seed(seed)
    d = torch.randn(*shape, generator=g, dtype=torch.float64)
    # one pattern for every batch: torch's batched CSR needs equal nnz per batch
    d = d * (torch.rand(*shape[-2:], generator=g) < density)
    return d, (d.to_sparse_csr() if layout == 'csr' else d.to_sparse())


def _T(t):
    return paddle.Tensor(t)


@pytest.mark.parametrize('layout', ['coo', 'csr'])
@pytest.mark.parametrize('op', ['add', 'subtract', 'multiply'])
def test_elementwise_merges_patterns(op, layout):
    dx, x = _rand_sparse((6, 7), 0.4, 1, layout)
    dy, y = _rand_sparse((6, 7), 0.4, 2, layout)
    out = getattr(SP, op)(_T(x), _T(y))._t
    assert out.layout == x.layout
    ref = {'add': dx + dy, 'subtract': dx - dy, 'multiply': dx * dy}[op]
    torch.testing.assert_close(out.to_dense(), ref)
    if op == 'multiply':   # intersection only
        assert out.to_sparse_coo()._nnz() == int(((dx != 0) & (dy != 0)).sum())


def test_elementwise_batched_and_dense_dims():
    dx, x = _rand_sparse((2, 5, 4), 0.5, 3)
    dy, y = _rand_sparse((2, 5, 4), 0.5, 4)
    torch.testing.assert_close(SP.add(_T(x), _T(y))._t.to_dense(), dx + dy)
    # hybrid COO: sparse (N, L) + dense channel
    vals = torch.randn(3, 4, dtype=torch.float64)
    a = torch.sparse_coo_tensor(torch.tensor([[0, 1, 1], [2, 0, 3]]), vals, (2, 4, 4))
    b = torch.sparse_coo_tensor(torch.tensor([[1, 1], [0, 1]]), vals[:2], (2, 4, 4))
    torch.testing.assert_close(SP.subtract(_T(a), _T(b))._t.to_dense(), a.to_dense() - b.to_dense())


@pytest.mark.parametrize('layout', ['coo', 'csr'])
@pytest.mark.parametrize('batched', [False, True])
def test_spmm_and_grads(layout, batched):
    shape = (3, 8, 10) if batched else (8, 10)
    dx, x = _rand_sparse(shape, 0.3, 5, layout)
    y = torch.randn(*(shape[:-2] + (10, 6)), dtype=torch.float64, requires_grad=True)
    out = SP.matmul(_T(x), _T(y))._t
    torch.testing.assert_close(out, dx @ y)
    out.sum().backward()
    torch.testing.assert_close(y.grad, dx.transpose(-1, -2) @ torch.ones_like(out))
    # gradient w.r.t. the stored values: d sum(A @ Y) / dA_ik = sum_j Y_kj at the stored coordinates
    coo = (x.to_sparse_coo() if layout == 'csr' else x).coalesce()
    vals = coo.values().clone().requires_grad_(True)
    xs = torch.sparse_coo_tensor(coo.indices(), vals, coo.shape)
    SP.matmul(_T(xs), _T(y.detach()))._t.sum().backward()
    rowsum = y.detach().sum(-1)
    idx = coo.indices()
    want = rowsum[idx[0], idx[2]] if batched else rowsum[idx[1]]
    torch.testing.assert_close(vals.grad, want)


def test_mv_dense_sparse_and_addmm():
    dx, x = _rand_sparse((7, 5), 0.5, 6, 'csr')
    v = torch.randn(5, dtype=torch.float64)
    torch.testing.assert_close(SP.mv(_T(x), _T(v))._t, dx @ v)
    a = torch.randn(4, 7, dtype=torch.float64)
    torch.testing.assert_close(SP.matmul(_T(a), _T(x))._t, a @ dx)
    inp = torch.randn(7, 3, dtype=torch.float64)
    y = torch.randn(5, 3, dtype=torch.float64)
    torch.testing.assert_close(SP.addmm(_T(inp), _T(x), _T(y), beta=0.5, alpha=2.0)._t, 0.5 * inp + 2.0 * dx @ y)


@pytest.mark.parametrize('batched', [False, True])
def test_spgemm(batched):
    sa = (2, 6, 9) if batched else (6, 9)
    sb = (2, 9, 5) if batched else (9, 5)
    da, a = _rand_sparse(sa, 0.3, 7, 'csr')
    db, b = _rand_sparse(sb, 0.3, 8, 'csr')
    out = SP.matmul(_T(a), _T(b))._t
    assert out.layout == torch.sparse_csr
    torch.testing.assert_close(out.to_dense(), da @ db)
    # empty product
    z = torch.zeros(9, 5, dtype=torch.float64).to_sparse_csr()
    if not batched:
        assert SP.matmul(_T(a), _T(z))._t.to_dense().abs().sum() == 0


def test_masked_matmul_sddmm():
    x = torch.randn(2, 6, 16, dtype=torch.float64, requires_grad=True)
    y = torch.randn(2, 16, 7, dtype=torch.float64)
    dm, mask = _rand_sparse((2, 6, 7), 0.4, 9, 'csr')
    out = SP.masked_matmul(_T(x), _T(y), _T(mask))._t
    assert out.layout == torch.sparse_csr
    torch.testing.assert_close(out.to_dense(), (x @ y) * (dm != 0))
    out.values().sum().backward()
    torch.testing.assert_close(x.grad, ((dm != 0).double()) @ y.transpose(1, 2))


def test_transpose_and_softmax():
    dx, x = _rand_sparse((2, 5, 6), 0.5, 10)
    torch.testing.assert_close(SP.transpose(_T(x), [0, 2, 1])._t.to_dense(), dx.transpose(1, 2))
    with pytest.raises(ValueError):
        SP.transpose(_T(torch.sparse_coo_tensor(torch.tensor([[0]]), torch.ones(1, 3), (2, 3))), [1, 0])
    dm, m = _rand_sparse((4, 6), 0.5, 11, 'csr')
    sm = SN.functional.softmax(_T(m))._t.to_dense()
    for r in range(4):
        nz = dm[r] != 0
        if nz.any():
            torch.testing.assert_close(sm[r, nz], torch.softmax(dm[r, nz], 0))


def test_sparse_attention_with_masks_and_grads():
    torch.manual_seed(0)
    B, H, S, D = 2, 2, 8, 16
    q, k, v = (torch.randn(B, H, S, D, dtype=torch.float64, requires_grad=True) for _ in range(3))
    pat = (torch.rand(B * H, S, S) < 0.5) | torch.eye(S, dtype=torch.bool)
    pat_coo = pat.double().to_sparse()   # per-head patterns differ in nnz: COO storage
    kpm = torch.ones(B, S)
    kpm[1, -3:] = 0
    am = torch.tril(torch.ones(S, S))
    out = SN.functional.attention(_T(q), _T(k), _T(v), _T(pat_coo),
                                  key_padding_mask=_T(kpm), attn_mask=_T(am))._t
    s = q @ k.transpose(-1, -2) / D ** 0.5
    keep = pat.view(B, H, S, S) & (kpm.view(B, 1, 1, S) != 0) & (am.view(1, 1, S, S) != 0)
    ref = torch.nan_to_num(torch.softmax(s.masked_fill(~keep, float('-inf')), -1)) @ v
    torch.testing.assert_close(out, ref)
    g = torch.randn_like(out)
    gs = torch.autograd.grad(out, (q, k, v), g)
    gr = torch.autograd.grad(ref, (q, k, v), g)
    for a, b in zip(gs, gr):
        torch.testing.assert_close(a, b)
