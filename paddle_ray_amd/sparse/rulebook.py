"""Sparse 3-D convolution and pooling on active sites only (parity: the reference's sparse conv
kernels paddle/phi/kernels/sparse/gpu/conv_kernel.cu + conv.cu.h rulebook, and
python/paddle/sparse/nn/functional/conv.py / pooling.py).

Gather - GEMM - scatter: a RULEBOOK lists, for every kernel offset k, the (input site, output site)
pairs it connects; the output of offset k is ``feats[in] @ W[k]`` scatter-added into ``out``. Sites
are found by hashing coordinates to int64 keys (sorted + binary search), so memory and work are
O(nnz x kernel volume) -- never the dense N x D x H x W grid. A regular conv activates every output
site reached by an active input; a submanifold conv keeps exactly the input's active sites.
Features are [nnz, C] (NDHWC COO with the channel as the dense dim); everything is differentiable
through index_select / mm / index_add (the GEMMs are the framework's on the device).
"""
import itertools

import torch


def _triple(v):
    return (v, v, v) if isinstance(v, int) else tuple(v)


def _key(c, dims):
    """(n, d, h, w) int64 coords [P, 4] -> linear keys on a grid of ``dims`` = (N, D, H, W)."""
    N, D, H, W = dims
    return ((c[:, 0] * D + c[:, 1]) * H + c[:, 2]) * W + c[:, 3]


def out_spatial(in_sp, kernel, stride, padding, dilation):
    return tuple((i + 2 * p - d * (k - 1) - 1) // s + 1
                 for i, k, s, p, d in zip(in_sp, kernel, stride, padding, dilation))


def build_rulebook(coords, batch, in_sp, kernel, stride, padding, dilation, subm):
    """coords [nnz, 4] int64 (n, d, h, w). Returns (out_coords [m, 4], out spatial dims,
    [(k, in_idx, out_idx)] per kernel offset with at least one pair)."""
    kernel, stride, padding, dilation = (_triple(v) for v in (kernel, stride, padding, dilation))
    dev = coords.device
    if subm:
        stride = (1, 1, 1)
        padding = tuple(d * (k - 1) // 2 for d, k in zip(dilation, kernel))
        osp = tuple(in_sp)
    else:
        osp = out_spatial(in_sp, kernel, stride, padding, dilation)
    offs = torch.tensor(list(itertools.product(*[range(k) for k in kernel])), dtype=torch.int64, device=dev)
    K, P = offs.shape[0], coords.shape[0]
    st = torch.tensor(stride, device=dev)
    num = coords[None, :, 1:] + torch.tensor(padding, device=dev) - offs[:, None, :] * torch.tensor(dilation, device=dev)
    ok = (num % st == 0).all(-1)
    o = torch.div(num, st, rounding_mode='floor')
    ok &= ((o >= 0) & (o < torch.tensor(osp, device=dev))).all(-1)          # [K, P]
    kk, ii = ok.nonzero(as_tuple=True)
    oc = torch.cat([coords[ii, :1], o[kk, ii]], 1)                           # candidate outputs
    dims = (batch,) + osp
    keys = _key(oc, dims)
    if subm:
        in_keys = _key(coords, (batch,) + tuple(in_sp))
        sk, order = torch.sort(in_keys)
        pos = torch.searchsorted(sk, keys).clamp(max=max(P - 1, 0))
        hit = sk[pos] == keys if P else torch.zeros_like(keys, dtype=torch.bool)
        kk, ii, oidx = kk[hit], ii[hit], order[pos[hit]]
        out_coords = coords
    else:
        uk, oidx = torch.unique(keys, return_inverse=True)
        W_, H_, D_ = osp[2], osp[1], osp[0]
        out_coords = torch.stack([uk // (D_ * H_ * W_), (uk // (H_ * W_)) % D_, (uk // W_) % H_, uk % W_], 1)
    rules = []
    for k in range(K):
        sel = kk == k
        if bool(sel.any()):
            rules.append((k, ii[sel], oidx[sel]))
    return out_coords, osp, rules


def sparse_conv3d(feats, coords, batch, in_sp, weight, bias, stride, padding, dilation, groups, subm):
    """feats [nnz, Cin]; weight [kD, kH, kW, Cin/groups, Cout]. Returns (out_feats, out_coords,
    out spatial dims)."""
    kD, kH, kW, cin_g, cout = weight.shape
    out_coords, osp, rules = build_rulebook(coords, batch, in_sp, (kD, kH, kW), stride, padding, dilation, subm)
    w = weight.reshape(kD * kH * kW, cin_g, cout)
    out = feats.new_zeros((out_coords.shape[0], cout))
    cout_g = cout // groups
    for k, ii, oo in rules:
        x = feats.index_select(0, ii)
        if groups == 1:
            y = x @ w[k]
        else:
            y = torch.cat([x[:, g * cin_g:(g + 1) * cin_g] @ w[k][:, g * cout_g:(g + 1) * cout_g]
                           for g in range(groups)], 1)
        out = out.index_add(0, oo, y.to(out.dtype))
    if bias is not None:
        out = out + bias
    return out, out_coords, osp


def sparse_max_pool3d(feats, coords, batch, in_sp, kernel, stride, padding):
    """Max over the ACTIVE input sites of each window; windows without one stay inactive."""
    kernel = _triple(kernel)
    stride = _triple(stride) if stride is not None else kernel
    out_coords, osp, rules = build_rulebook(coords, batch, in_sp, kernel, stride, padding, (1, 1, 1), False)
    C = feats.shape[1]
    out = torch.full((out_coords.shape[0], C), float('-inf'), dtype=feats.dtype, device=feats.device)
    ii = torch.cat([r[1] for r in rules]) if rules else torch.zeros(0, dtype=torch.int64, device=feats.device)
    oo = torch.cat([r[2] for r in rules]) if rules else ii
    out = out.scatter_reduce(0, oo[:, None].expand(-1, C), feats.index_select(0, ii), 'amax', include_self=False)
    return out, out_coords, osp
