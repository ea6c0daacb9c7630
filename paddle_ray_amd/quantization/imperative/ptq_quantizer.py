"""Calibration quantizers for post-training quantization (parity:
python/paddle/quantization/imperative/ptq_quantizer.py, static/quantization/
cal_kl_threshold.py)."""
import abc
import math

import numpy as np
import torch

from ...framework.core import _u


def _np(t):
    return _u(t).detach().float().cpu().numpy() if hasattr(t, '_t') or torch.is_tensor(t) \
        else np.asarray(t, np.float32)


def cal_kl_threshold(hist, bin_width, bits):
    """KL-divergence calibration (TensorRT method): the clipping threshold whose quantized
    distribution is closest to the reference histogram."""
    hist = np.asarray(hist, np.float64)
    n_bins = hist.size
    quant_range = 2 ** (bits - 1) - 1
    # search the upper half only: bounds the clipping to at most 2x (sparse calibration
    # histograms otherwise favour degenerate tiny thresholds)
    start = max(quant_range + 1, n_bins // 2)
    best_kl, best_i = np.inf, n_bins
    total = hist.sum()
    if total == 0:
        return n_bins * bin_width
    for i in range(start, n_bins + 1):
        p = hist[:i].copy()
        p[i - 1] += hist[i:].sum()
        # quantize the first i bins into quant_range+1 levels
        idx = (np.arange(i) * (quant_range + 1) // i)
        q = np.zeros(i)
        for lvl in range(quant_range + 1):
            m = idx == lvl
            nz = m & (hist[:i] != 0)
            if nz.any():
                q[nz] = hist[:i][m].sum() / nz.sum()
        pn, qn = p / max(p.sum(), 1e-12), q / max(q.sum(), 1e-12)
        mask = pn > 0
        if (qn[mask] == 0).any():
            kl = np.inf
        else:
            kl = float(np.sum(pn[mask] * np.log(pn[mask] / qn[mask])))
        if kl < best_kl:
            best_kl, best_i = kl, i
    return (best_i + 0.5) * bin_width


class BaseQuantizer(metaclass=abc.ABCMeta):
    def __init__(self, quant_bits=8):
        self.quant_bits = quant_bits
        self.abs_max_vals = []
        self.thresholds = []

    @abc.abstractmethod
    def sample_data(self, layer, tensors):
        ...

    @abc.abstractmethod
    def cal_thresholds(self):
        ...


class AbsmaxQuantizer(BaseQuantizer):
    """Per-tensor running max |x| for every observed tensor."""

    def sample_data(self, layer, tensors):
        vals = [float(np.abs(_np(t)).max()) if np.size(_np(t)) else 0.0 for t in tensors]
        self.abs_max_vals = vals if not self.abs_max_vals else \
            [max(a, b) for a, b in zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = self.abs_max_vals


class PerChannelAbsmaxQuantizer(BaseQuantizer):
    """Per-output-channel max |w| (axis 0 for conv weights, axis 1 for linear weights)."""

    def sample_data(self, layer, tensors):
        from ... import nn
        axis = 1 if isinstance(layer, nn.Linear) else 0
        vals = []
        for t in tensors:
            a = np.abs(_np(t))
            dims = tuple(d for d in range(a.ndim) if d != axis)
            vals.append(list(a.max(axis=dims)) if a.ndim > 1 else [float(a.max())])
        if not self.abs_max_vals:
            self.abs_max_vals = vals
        else:
            self.abs_max_vals = [list(np.maximum(a, b)) for a, b in zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = self.abs_max_vals


class _HistBase(BaseQuantizer):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64):
        super().__init__(quant_bits)
        self.bins, self.upsample_bins = bins, upsample_bins
        self.hists = []

    def sample_data(self, layer, tensors):
        arrays = [np.abs(_np(t)).ravel() for t in tensors]
        if not self.hists:
            self.abs_max_vals = [float(a.max()) if a.size else 0.0 for a in arrays]
            self.hists = [np.histogram(a, bins=self.bins, range=(0, m or 1.0))[0]
                          .astype(np.float64) for a, m in zip(arrays, self.abs_max_vals)]
            return
        for i, a in enumerate(arrays):
            m = float(a.max()) if a.size else 0.0
            if m > self.abs_max_vals[i]:  # re-bin the old histogram onto the wider range
                old = self.hists[i]
                centers = (np.arange(self.bins) + 0.5) * self.abs_max_vals[i] / self.bins
                self.hists[i] = np.histogram(centers, bins=self.bins, range=(0, m),
                                             weights=old)[0]
                self.abs_max_vals[i] = m
            self.hists[i] += np.histogram(a, bins=self.bins, range=(0, self.abs_max_vals[i]
                                                                    or 1.0))[0]


class KLQuantizer(_HistBase):
    def cal_thresholds(self):
        self.thresholds = [cal_kl_threshold(h, (m or 1.0) / self.bins, self.quant_bits)
                           for h, m in zip(self.hists, self.abs_max_vals)]


class HistQuantizer(_HistBase):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64, hist_percent=0.99999):
        super().__init__(quant_bits, bins, upsample_bins)
        self.hist_percent = hist_percent

    def cal_thresholds(self):
        out = []
        for h, m in zip(self.hists, self.abs_max_vals):
            c = np.cumsum(h) / max(h.sum(), 1e-12)
            i = int(np.searchsorted(c, self.hist_percent))
            out.append((i + 0.5) * (m or 1.0) / self.bins)
        self.thresholds = out


SUPPORT_ACT_QUANTIZERS = [AbsmaxQuantizer, HistQuantizer, KLQuantizer]
SUPPORT_WT_QUANTIZERS = [AbsmaxQuantizer, PerChannelAbsmaxQuantizer]
