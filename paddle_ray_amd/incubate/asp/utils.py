"""n:m structured-sparsity masks (parity: python/paddle/incubate/asp/utils.py).

``n:m`` means at least ``n`` zeros in every group of ``m`` consecutive weights of a row
(1D), or in every row AND column of each m x m block (2D). 2:4 is the pattern the CDNA4
sparse matrix cores (``v_smfmac``) consume. Masks keep the largest-magnitude weights.
"""
import itertools
from enum import Enum

import numpy as np

__all__ = []


class MaskAlgo(Enum):
    MASK_1D = 'get_mask_1d'
    MASK_2D_GREEDY = 'get_mask_2d_greedy'
    MASK_2D_BEST = 'get_mask_2d_best'


class CheckMethod(Enum):
    CHECK_1D = 'check_mask_1d'
    CHECK_2D = 'check_mask_2d'

    @staticmethod
    def get_checking_method(mask_algo):
        assert isinstance(mask_algo, MaskAlgo), "mask_algo should be MaskAlgo type"
        return CheckMethod.CHECK_1D if mask_algo == MaskAlgo.MASK_1D else CheckMethod.CHECK_2D


def calculate_density(x):
    x = np.asarray(x).reshape(-1)
    return float(np.count_nonzero(x)) / x.size


def _pad_cols(mat, m):
    r = mat.shape[1] % m
    if r:
        mat = np.concatenate([mat, np.zeros((mat.shape[0], m - r), mat.dtype)], axis=1)
    return mat


def _as_2d(mat):
    mat = np.asarray(mat)
    return mat.reshape(1, -1) if mat.ndim <= 1 else mat


def check_mask_1d(mat, n, m):
    groups = _pad_cols(_as_2d(mat), m).reshape(-1, m)
    return bool((np.count_nonzero(groups, axis=1) <= m - n).all())


def get_mask_1d(mat, n, m):
    """Keep the m-n largest |values| of every 1 x m group."""
    mat = _as_2d(mat)
    rows, cols = mat.shape
    groups = np.abs(_pad_cols(mat, m).reshape(-1, m))
    keep = np.argsort(-groups, axis=1, kind='stable')[:, :m - n]
    mask = np.zeros_like(groups, dtype=np.float32)
    np.put_along_axis(mask, keep, 1.0, axis=1)
    return mask.reshape(rows, -1)[:, :cols]


def _blocks_2d(mat, m):
    mat = _as_2d(mat)
    h, w = mat.shape
    ph, pw = (-h) % m, (-w) % m
    padded = np.pad(mat, ((0, ph), (0, pw)))
    H, W = padded.shape
    return padded.reshape(H // m, m, W // m, m).transpose(0, 2, 1, 3), (h, w)


def _unblock(blocks, hw):
    bh, bw, m, _ = blocks.shape
    return blocks.transpose(0, 2, 1, 3).reshape(bh * m, bw * m)[:hw[0], :hw[1]]


def check_mask_2d(mat, n, m):
    blocks, _ = _blocks_2d(mat, m)
    nz = blocks != 0
    return bool((nz.sum(axis=3) <= m - n).all() and (nz.sum(axis=2) <= m - n).all())


def get_mask_2d_greedy(mat, n, m):
    """Per m x m block: take entries by descending |value| while their row and column
    still have fewer than m-n kept entries."""
    blocks, hw = _blocks_2d(mat, m)
    mask = np.zeros(blocks.shape, np.float32)
    for bi in range(blocks.shape[0]):
        for bj in range(blocks.shape[1]):
            b = np.abs(blocks[bi, bj])
            rc, cc = np.zeros(m, int), np.zeros(m, int)
            for flat in np.argsort(-b, axis=None, kind='stable'):
                r, c = divmod(int(flat), m)
                if rc[r] < m - n and cc[c] < m - n:
                    mask[bi, bj, r, c] = 1.0
                    rc[r] += 1
                    cc[c] += 1
    return _unblock(mask, hw)


_PATTERNS = {}


def _compute_valid_2d_patterns(n, m):
    """All m x m 0/1 patterns with exactly m-n ones per row and per column."""
    key = (n, m)
    if key not in _PATTERNS:
        rows = [r for r in itertools.product([0, 1], repeat=m) if sum(r) == m - n]
        pats = [np.array(p, np.float32) for p in itertools.product(rows, repeat=m)
                if all(sum(col) == m - n for col in zip(*p))]
        _PATTERNS[key] = np.stack(pats)
    return _PATTERNS[key]


def get_mask_2d_best(mat, n, m):
    """Per m x m block: the valid pattern that keeps the largest total |value|."""
    blocks, hw = _blocks_2d(mat, m)
    pats = _compute_valid_2d_patterns(n, m)  # [P, m, m]
    flat = np.abs(blocks).reshape(-1, m * m)
    best = np.argmax(flat @ pats.reshape(len(pats), -1).T, axis=1)
    mask = pats[best].reshape(blocks.shape)
    return _unblock(mask, hw)


def _to_2d(t):
    shape = t.shape
    if t.ndim == 1:
        return t.reshape(1, -1), lambda x: x.reshape(shape)
    if t.ndim == 2:
        return t, lambda x: x
    if t.ndim == 3:
        return t.reshape(-1, shape[2]), lambda x: x.reshape(shape)
    if t.ndim == 4:  # prune along axis 2 (the reduction channel after the caller's .T)
        p = t.transpose(0, 1, 3, 2)
        return p.reshape(-1, shape[2]), \
            lambda x: x.reshape(shape[0], shape[1], shape[3], shape[2]).transpose(0, 1, 3, 2)
    raise ValueError(f"tensors of rank {t.ndim} are not supported")


def create_mask(tensor, func_name=MaskAlgo.MASK_1D, n=2, m=4):
    t = np.asarray(tensor)
    func = globals()[(func_name if isinstance(func_name, MaskAlgo) else MaskAlgo(func_name)).value]
    mat, back = _to_2d(t.astype(np.float32))
    return back(func(mat, n, m)).astype(t.dtype)


def check_sparsity(tensor, func_name=CheckMethod.CHECK_1D, n=2, m=4):
    t = np.asarray(tensor)
    func = globals()[(func_name if isinstance(func_name, CheckMethod)
                      else CheckMethod(func_name)).value]
    mat, _ = _to_2d(t)
    return func(mat, n, m)
