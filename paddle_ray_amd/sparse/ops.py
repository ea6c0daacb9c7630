"""Sparse kernels written as index math over COO coordinates (parity: the reference's sparse phi
kernels paddle/phi/kernels/sparse/gpu/{elementwise_kernel.cu, matmul_kernel.cu,
mask_kernel.cu, softmax_kernel.cu, fused_attention_kernel.cu} and
python/paddle/sparse/{binary,multiary}.py, sparse/nn/functional/{activation,transformer}.py).

Storage stays the PyTorch sparse COO / CSR tensor (CSR is handled through its COO coordinates);
every op below computes on (indices, values) directly, O(nnz) memory and work, never a dense
grid, and is differentiable w.r.t. the values and the dense operands through
index_select / index_add / scatter_reduce:

* elementwise add / subtract / divide merge the two patterns (union of coordinates, missing
  entries read as 0); multiply keeps the intersection.
* SpMM (sparse @ dense): gather the dense rows named by the column coordinate, scale by the
  value, segment-sum into the output row.
* SpGEMM (sparse @ sparse): expand - sort - compress. Each A entry (i, k) is expanded against
  B's row k (row pointers from a bincount of B's keys), products are keyed by (i, j) and summed.
* SDDMM (masked_matmul): one dot product per mask coordinate.
* row softmax: segment max (scatter_reduce amax) / exp / segment sum over the stored entries.
* sparse attention: SDDMM of q.k on the mask pattern, padding / attention masks applied on those
  entries, row softmax, SpMM with v -- O(nnz * head_dim) instead of O(S^2).

Batched operands carry a leading batch coordinate (3-D COO / batched CSR): rows are keyed by
(batch, row) so the same code serves 2-D and 3-D.
"""
import torch


def _prod(v):
    p = 1
    for x in v:
        p *= int(x)
    return p


def coo_parts(t):
    """(indices [sparse_dim, nnz], values [nnz, *dense], shape, layout) of a coalesced view."""
    layout = t.layout
    if layout == torch.sparse_csr:
        t = t.to_sparse_coo()
    elif layout != torch.sparse_coo:
        raise TypeError(f"expected a sparse COO / CSR tensor, got layout {layout}")
    t = t.coalesce()
    return t.indices(), t.values(), tuple(t.shape), layout


def make(idx, vals, shape, layout, coalesced=False):
    """Build a sparse tensor of ``layout`` from COO parts (CSR for 2-D / batched 3-D)."""
    t = torch.sparse_coo_tensor(idx, vals, shape, is_coalesced=coalesced)
    if not coalesced:
        t = t.coalesce()
    if layout == torch.sparse_csr and idx.shape[0] in (2, 3) and vals.dim() == 1:
        if idx.shape[0] == 2:
            return t.to_sparse_csr()
        return _batched_csr(t, shape)
    return t


def _batched_csr(t, shape):
    """Batched CSR from a coalesced 3-D COO (torch stores batched CSR with the same nnz in every
    batch; other patterns stay COO)."""
    B, M = int(shape[0]), int(shape[1])
    idx, v = t.indices(), t.values()
    per = torch.bincount(idx[0], minlength=B)
    if idx.shape[1] and bool((per != per[0]).any()):
        return t
    n = idx.shape[1] // max(B, 1)
    rows = torch.bincount(idx[0] * M + idx[1], minlength=B * M).view(B, M)
    crow = torch.cat([rows.new_zeros(B, 1), torch.cumsum(rows, 1)], 1)
    return torch.sparse_csr_tensor(crow, idx[2].view(B, n), v.view(B, n), tuple(shape))


def linear_keys(idx, dims):
    """Row-major linearisation of coordinates ``idx`` [d, nnz] over ``dims``."""
    k = torch.zeros(idx.shape[1], dtype=torch.int64, device=idx.device)
    for d, n in enumerate(dims):
        k = k * int(n) + idx[d]
    return k


def unravel(keys, dims):
    out = []
    for n in reversed(dims):
        out.append(keys % int(n))
        keys = keys // int(n)
    return torch.stack(out[::-1]) if out else keys[None, :0]


# ----------------------------------------------------------------------------- elementwise

def elementwise(op, x, y):
    """x (op) y for two sparse tensors of one shape and layout."""
    ix, vx, shape, layout = coo_parts(x)
    iy, vy, shape_y, layout_y = coo_parts(y)
    if shape != shape_y:
        raise ValueError(f"sparse {op}: shapes {list(shape)} and {list(shape_y)} differ")
    if ix.shape[0] != iy.shape[0]:
        raise ValueError(f"sparse {op}: operands have different sparse dims")
    sd = ix.shape[0]
    dims = shape[:sd]
    kx, ky = linear_keys(ix, dims), linear_keys(iy, dims)
    uk, inv = torch.unique(torch.cat([kx, ky]), return_inverse=True)
    nx = kx.numel()
    dt = torch.promote_types(vx.dtype, vy.dtype)
    dense = tuple(vx.shape[1:])
    ax = vx.new_zeros((uk.numel(),) + dense, dtype=dt).index_add(0, inv[:nx], vx.to(dt))
    ay = vy.new_zeros((uk.numel(),) + dense, dtype=dt).index_add(0, inv[nx:], vy.to(dt))
    if op == 'multiply':
        hx = torch.zeros(uk.numel(), dtype=torch.bool, device=uk.device)
        hy = hx.clone()
        hx[inv[:nx]] = True
        hy[inv[nx:]] = True
        keep = (hx & hy).nonzero().squeeze(1)
        uk, ax, ay = uk[keep], ax[keep], ay[keep]
        vals = ax * ay
    elif op == 'add':
        vals = ax + ay
    elif op == 'subtract':
        vals = ax - ay
    elif op == 'divide':
        vals = ax / ay
    else:
        raise ValueError(op)
    return make(unravel(uk, dims), vals, shape, layout, coalesced=True)


# ----------------------------------------------------------------------------- products

def _rows_cols(idx, shape):
    """(batch, row, col) coordinate vectors of a 2-D or batched 3-D sparse matrix."""
    if idx.shape[0] == 2:
        return torch.zeros_like(idx[0]), idx[0], idx[1], 1
    if idx.shape[0] == 3:
        return idx[0], idx[1], idx[2], shape[0]
    raise ValueError("sparse matmul expects a 2-D or batched 3-D sparse matrix")


def spmm(x, dense):
    """sparse [B?, M, K] @ dense [B?, K, N] -> dense [B?, M, N]."""
    idx, v, shape, _ = coo_parts(x)
    b, i, k, B = _rows_cols(idx, shape)
    M, K = shape[-2], shape[-1]
    vec = dense.dim() == len(shape) - 1
    d = dense.unsqueeze(-1) if vec else dense
    if d.shape[-2] != K:
        raise ValueError(f"sparse matmul: inner dims {K} and {d.shape[-2]} differ")
    N = d.shape[-1]
    dt = torch.promote_types(v.dtype, d.dtype)
    rows = d.reshape(-1, K, N).expand(B, K, N).reshape(B * K, N).to(dt)
    src = rows.index_select(0, b * K + k) * v.to(dt).unsqueeze(1)
    out = src.new_zeros(B * M, N).index_add(0, b * M + i, src)
    out = out.view(B, M, N) if len(shape) == 3 else out.view(M, N)
    return out.squeeze(-1) if vec else out


def dense_spmm(dense, y):
    """dense [B?, M, K] @ sparse [B?, K, N] -> dense [B?, M, N] (column scatter)."""
    idx, v, shape, _ = coo_parts(y)
    b, k, j, B = _rows_cols(idx, shape)
    K, N = shape[-2], shape[-1]
    M = dense.shape[-2]
    dt = torch.promote_types(v.dtype, dense.dtype)
    cols = dense.reshape(-1, M, K).expand(B, M, K).transpose(1, 2).reshape(B * K, M).to(dt)
    src = cols.index_select(0, b * K + k) * v.to(dt).unsqueeze(1)          # [nnz, M]
    out = src.new_zeros(B * N, M).index_add(0, b * N + j, src)
    out = out.view(B, N, M).transpose(1, 2)
    return out if len(shape) == 3 else out[0]


def spgemm(x, y):
    """sparse [B?, M, K] @ sparse [B?, K, N] -> sparse (layout of x), expand-sort-compress."""
    ia, va, sa, layout = coo_parts(x)
    ib, vb, sb, _ = coo_parts(y)
    ba, i, ka, B = _rows_cols(ia, sa)
    bb, kb, j, _ = _rows_cols(ib, sb)
    M, K, N = sa[-2], sa[-1], sb[-1]
    if sb[-2] != K:
        raise ValueError(f"sparse matmul: inner dims {K} and {sb[-2]} differ")
    rowb = bb * K + kb                                  # B is coalesced: sorted by (b, k, j)
    cnt = torch.bincount(rowb, minlength=B * K)
    start = torch.cumsum(cnt, 0) - cnt
    keya = ba * K + ka
    c = cnt[keya]                                       # products contributed by each A entry
    total = int(c.sum())
    dt = torch.promote_types(va.dtype, vb.dtype)
    if total == 0:
        idx = ia.new_zeros((ia.shape[0], 0))
        return make(idx, va.new_zeros(0, dtype=dt), sa[:-1] + (N,), layout, coalesced=True)
    rep = torch.repeat_interleave(torch.arange(ia.shape[1], device=ia.device), c)
    first = torch.cumsum(c, 0) - c
    pos = start[keya][rep] + torch.arange(total, device=ia.device) - first[rep]
    vals = va.to(dt)[rep] * vb.to(dt)[pos]
    key = (ba[rep] * M + i[rep]) * N + j[pos]
    uk, inv = torch.unique(key, return_inverse=True)
    out = vals.new_zeros(uk.numel()).index_add(0, inv, vals)
    dims = (B, M, N) if len(sa) == 3 else (M, N)   # 2-D: batch coordinate is 0, keys < M*N
    return make(unravel(uk, dims), out, dims, layout, coalesced=True)


def sddmm(x, y, mask):
    """(x @ y) sampled at ``mask``'s coordinates -> sparse with mask's pattern and layout."""
    idx, _, shape, layout = coo_parts(mask)
    b, i, j, B = _rows_cols(idx, shape)
    M, N = shape[-2], shape[-1]
    K = x.shape[-1]
    dt = torch.promote_types(x.dtype, y.dtype)
    xr = x.reshape(-1, M, K).expand(B, M, K).reshape(B * M, K).to(dt)
    yc = y.reshape(-1, K, N).expand(B, K, N).transpose(1, 2).reshape(B * N, K).to(dt)
    ra, rb = b * M + i, b * N + j
    nnz = idx.shape[1]
    step = max(1, (1 << 26) // max(1, K))               # bound the gathered [chunk, K] operands
    vals = torch.cat([(xr.index_select(0, ra[s:s + step]) * yc.index_select(0, rb[s:s + step])).sum(-1)
                      for s in range(0, nnz, step)]) if nnz else xr.new_zeros(0)
    return make(idx, vals, shape, layout, coalesced=True)


# ----------------------------------------------------------------------------- softmax / attention

def _segment_softmax(scores, seg, nseg):
    """Softmax of ``scores`` within each segment id of ``seg``; all -inf segments -> 0."""
    mx = torch.full((nseg,), float('-inf'), dtype=scores.dtype, device=scores.device)
    mx = mx.scatter_reduce(0, seg, scores.detach(), 'amax', include_self=True)
    mx = torch.where(torch.isfinite(mx), mx, torch.zeros_like(mx))
    e = torch.exp(scores - mx[seg])
    den = e.new_zeros(nseg).index_add(0, seg, e)
    return e / den[seg].clamp_min(torch.finfo(e.dtype).tiny)


def row_softmax(x):
    """Softmax over the stored entries of every row (last axis) of a sparse tensor."""
    idx, v, shape, layout = coo_parts(x)
    if v.dim() != 1:
        raise ValueError("sparse softmax expects scalar values (no dense dims)")
    seg = linear_keys(idx[:-1], shape[:-1])
    return make(idx, _segment_softmax(v, seg, _prod(shape[:-1])), shape, layout, coalesced=True)


def attention(q, k, v, mask, key_padding_mask=None, attn_mask=None):
    """softmax(q k^T / sqrt(d)) v on the coordinates of ``mask`` ([B*H, S, S] sparse);
    q/k/v [B, H, S, D]. ``key_padding_mask`` [B, S] and ``attn_mask`` [S, S] drop (==0) entries."""
    B, H, S, D = q.shape
    idx, _, shape, _ = coo_parts(mask)
    if idx.shape[0] == 2:                               # one [S, S] pattern shared by all heads
        n = idx.shape[1]
        bh = torch.arange(B * H, device=idx.device).repeat_interleave(n)
        i, j = idx[0].repeat(B * H), idx[1].repeat(B * H)
    else:
        bh, i, j = idx[0], idx[1], idx[2]
        if shape[0] != B * H:
            raise ValueError(f"sparse attention: mask batch {shape[0]} != B*H = {B * H}")
    qf, kf, vf = (t.reshape(B * H * S, D) for t in (q, k, v))
    ri, rj = bh * S + i, bh * S + j
    s = (qf.index_select(0, ri) * kf.index_select(0, rj)).sum(-1) * (1.0 / D ** 0.5)
    drop = torch.zeros_like(s, dtype=torch.bool)
    if key_padding_mask is not None:
        kp = key_padding_mask.reshape(B, S)
        drop |= kp[bh // H, j] == 0
    if attn_mask is not None:
        drop |= attn_mask.reshape(S, S)[i, j] == 0
    s = s.masked_fill(drop, float('-inf'))
    sw = s.float() if s.dtype in (torch.float16, torch.bfloat16) else s   # softmax in >= fp32
    p = _segment_softmax(sw, ri, B * H * S).to(q.dtype)
    out = qf.new_zeros(B * H * S, D).index_add(0, ri, p.unsqueeze(1) * vf.index_select(0, rj))
    return out.view(B, H, S, D)
