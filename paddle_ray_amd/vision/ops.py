"""paddle.vision.ops: detection / region operators (parity: python/paddle/vision/ops.py —
yolo_loss :51, yolo_box :262, prior_box :425, box_coder :572, deform_conv2d :742,
DeformConv2D :951, distribute_fpn_proposals :1151, read_file :1289, decode_jpeg :1334,
psroi_pool :1384, roi_pool :1504, roi_align :1628, ConvNormActivation :1796, nms :1853,
generate_proposals :2023, matrix_nms :2190).

Every operator is written as batched tensor math (gathers, masks, reductions) so it runs
on the device that holds its inputs, and is differentiable through autograd where the
reference op has a gradient (roi_align / roi_pool / psroi_pool / deform_conv2d /
yolo_loss / box_coder). Data-dependent selection (NMS family, proposal generation) keeps
its greedy loop on the host-side index set only.
"""
import math

import numpy as np
import torch
import torch.nn.functional as TF

from ..framework.core import Tensor, _u, _w
from ..nn import BatchNorm2D, Conv2D, ReLU, Sequential
from ..nn.layer.layers import Layer

__all__ = ['yolo_loss', 'yolo_box', 'prior_box', 'box_coder', 'deform_conv2d', 'DeformConv2D',
           'distribute_fpn_proposals', 'generate_proposals', 'read_file', 'decode_jpeg',
           'roi_pool', 'RoIPool', 'psroi_pool', 'PSRoIPool', 'roi_align', 'RoIAlign', 'nms',
           'matrix_nms', 'ConvNormActivation']


def _pair(v):
    return (int(v), int(v)) if isinstance(v, (int, np.integer)) else (int(v[0]), int(v[1]))


def _batch_index(boxes_num, n_rois, device):
    """Image index of every RoI from the per-image RoI counts."""
    if boxes_num is None:
        return torch.zeros(n_rois, dtype=torch.long, device=device)
    bn = _u(boxes_num).to(device=device, dtype=torch.long).reshape(-1)
    return torch.repeat_interleave(torch.arange(bn.numel(), device=device), bn)


# ----------------------------------------------------------------------------
# bilinear sampling helper (zero outside the image, per corner)
# ----------------------------------------------------------------------------
def _bilinear_dcn(img, b, y, x):
    """Deformable-conv sampling: points with y <= -1 or y >= H (same for x) are zero and
    each of the 4 corners outside the image contributes zero (no coordinate clamping)."""
    N, C, H, W = img.shape
    feat = img.permute(0, 2, 3, 1)
    valid = ((y > -1) & (y < H) & (x > -1) & (x < W)).to(img.dtype)
    y0f, x0f = y.floor(), x.floor()
    ly, lx = y - y0f, x - x0f
    y0, x0 = y0f.long(), x0f.long()
    out = 0
    for dy, wy in ((0, 1 - ly), (1, ly)):
        for dx, wx in ((0, 1 - lx), (1, lx)):
            yy, xx = y0 + dy, x0 + dx
            ok = ((yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)).to(img.dtype)
            v = feat[b, yy.clamp(0, H - 1), xx.clamp(0, W - 1)]
            out = out + v * (wy * wx * ok)[..., None]
    return out * valid[..., None]


def _bilinear(img, b, y, x):
    """img [N,C,H,W]; b, y, x broadcastable index/coordinate tensors -> [..., C].

    RoIAlign convention: points with y < -1 or y > H (same for x) give zero, otherwise the
    coordinate is clamped into the image before interpolating."""
    N, C, H, W = img.shape
    feat = img.permute(0, 2, 3, 1)  # [N,H,W,C]
    valid = (y >= -1) & (y <= H) & (x >= -1) & (x <= W)
    y = y.clamp(min=0)
    x = x.clamp(min=0)
    y0 = y.floor().long()
    x0 = x.floor().long()
    y0c = y0.clamp(max=H - 1)
    x0c = x0.clamp(max=W - 1)
    y1 = (y0 + 1).clamp(max=H - 1)
    x1 = (x0 + 1).clamp(max=W - 1)
    y = torch.where(y0 >= H - 1, y0c.to(y.dtype), y)
    x = torch.where(x0 >= W - 1, x0c.to(x.dtype), x)
    ly, lx = y - y0c, x - x0c
    hy, hx = 1 - ly, 1 - lx
    out = (feat[b, y0c, x0c] * (hy * hx)[..., None] + feat[b, y0c, x1] * (hy * lx)[..., None] +
           feat[b, y1, x0c] * (ly * hx)[..., None] + feat[b, y1, x1] * (ly * lx)[..., None])
    return out * valid[..., None].to(out.dtype)


# ----------------------------------------------------------------------------
# RoI operators
# ----------------------------------------------------------------------------
def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1,
              aligned=True, name=None):
    """Bilinear RoI pooling (Mask R-CNN): each of the ph x pw bins averages a grid of
    bilinear samples (``sampling_ratio`` per axis, adaptive ceil(roi/bin) when <= 0)."""
    xt, bt = _u(x), _u(boxes).to(_u(x).dtype)
    ph, pw = _pair(output_size)
    R = bt.shape[0]
    dev = xt.device
    bidx = _batch_index(boxes_num, R, dev)
    off = 0.5 if aligned else 0.0
    x1, y1 = bt[:, 0] * spatial_scale - off, bt[:, 1] * spatial_scale - off
    x2, y2 = bt[:, 2] * spatial_scale - off, bt[:, 3] * spatial_scale - off
    rw, rh = x2 - x1, y2 - y1
    if not aligned:
        rw, rh = rw.clamp(min=1.0), rh.clamp(min=1.0)
    bh, bw = rh / ph, rw / pw
    if sampling_ratio > 0:
        gh = torch.full((R,), sampling_ratio, device=dev, dtype=torch.long)
        gw = gh.clone()
    else:
        gh = torch.ceil(rh / ph).long().clamp(min=1)
        gw = torch.ceil(rw / pw).long().clamp(min=1)
    GH = int(gh.max()) if R else 1
    GW = int(gw.max()) if R else 1
    iy = torch.arange(GH, device=dev, dtype=xt.dtype)
    ix = torch.arange(GW, device=dev, dtype=xt.dtype)
    py = torch.arange(ph, device=dev, dtype=xt.dtype)
    px = torch.arange(pw, device=dev, dtype=xt.dtype)
    # sample coordinates [R, ph, GH] and [R, pw, GW]
    ys = y1[:, None, None] + py[None, :, None] * bh[:, None, None] + \
        (iy[None, None, :] + 0.5) * (bh / gh.to(xt.dtype))[:, None, None]
    xs = x1[:, None, None] + px[None, :, None] * bw[:, None, None] + \
        (ix[None, None, :] + 0.5) * (bw / gw.to(xt.dtype))[:, None, None]
    my = (iy[None, :] < gh[:, None]).to(xt.dtype)  # [R, GH]
    mx = (ix[None, :] < gw[:, None]).to(xt.dtype)
    Y = ys.reshape(R, ph * GH)[:, :, None].expand(R, ph * GH, pw * GW)
    X = xs.reshape(R, pw * GW)[:, None, :].expand(R, ph * GH, pw * GW)
    v = _bilinear(xt, bidx[:, None, None], Y, X)  # [R, ph*GH, pw*GW, C]
    C = xt.shape[1]
    v = v.reshape(R, ph, GH, pw, GW, C)
    w = (my[:, None, :, None, None, None] * mx[:, None, None, None, :, None])
    cnt = (gh * gw).to(xt.dtype).clamp(min=1)
    out = (v * w).sum(dim=(2, 4)) / cnt[:, None, None, None]
    return _w(out.permute(0, 3, 1, 2).contiguous())


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    """Max RoI pooling over integer-quantized bins (Fast R-CNN); empty bins give 0."""
    xt, bt = _u(x), _u(boxes)
    ph, pw = _pair(output_size)
    N, C, H, W = xt.shape
    R = bt.shape[0]
    dev = xt.device
    bidx = _batch_index(boxes_num, R, dev)
    rs = torch.round(bt.float() * spatial_scale).long()
    x1, y1, x2, y2 = rs[:, 0], rs[:, 1], rs[:, 2], rs[:, 3]
    rw = (x2 - x1 + 1).clamp(min=1).float()
    rh = (y2 - y1 + 1).clamp(min=1).float()
    bh, bw = rh / ph, rw / pw
    hh = torch.arange(H, device=dev)
    ww = torch.arange(W, device=dev)
    feat = xt[bidx]  # [R,C,H,W]
    out = xt.new_zeros(R, C, ph, pw)
    neg = torch.finfo(xt.dtype).min
    for i in range(ph):
        hs = (torch.floor(i * bh).long() + y1).clamp(0, H)
        he = (torch.ceil((i + 1) * bh).long() + y1).clamp(0, H)
        mh = (hh[None] >= hs[:, None]) & (hh[None] < he[:, None])  # [R,H]
        for j in range(pw):
            ws = (torch.floor(j * bw).long() + x1).clamp(0, W)
            we = (torch.ceil((j + 1) * bw).long() + x1).clamp(0, W)
            mw = (ww[None] >= ws[:, None]) & (ww[None] < we[:, None])
            m = (mh[:, :, None] & mw[:, None, :])[:, None]  # [R,1,H,W]
            v = torch.where(m, feat, torch.full_like(feat, neg)).amax(dim=(2, 3))
            empty = ~m.flatten(1).any(1)
            out[:, :, i, j] = torch.where(empty[:, None], torch.zeros_like(v), v)
    return _w(out)


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    """Position-sensitive average RoI pooling (R-FCN): output channel c of bin (i, j)
    averages input channel (c*ph + i)*pw + j over the bin."""
    xt, bt = _u(x), _u(boxes)
    ph, pw = _pair(output_size)
    N, C, H, W = xt.shape
    if C % (ph * pw):
        raise ValueError("input channels must be a multiple of output_size[0]*output_size[1]")
    oc = C // (ph * pw)
    R = bt.shape[0]
    dev = xt.device
    bidx = _batch_index(boxes_num, R, dev)
    b = bt.to(xt.dtype)
    x1 = torch.round(b[:, 0]) * spatial_scale
    y1 = torch.round(b[:, 1]) * spatial_scale
    x2 = (torch.round(b[:, 2]) + 1.0) * spatial_scale
    y2 = (torch.round(b[:, 3]) + 1.0) * spatial_scale
    rw = (x2 - x1).clamp(min=0.1)
    rh = (y2 - y1).clamp(min=0.1)
    bh, bw = rh / ph, rw / pw
    hh = torch.arange(H, device=dev)
    ww = torch.arange(W, device=dev)
    feat = xt[bidx].reshape(R, oc, ph, pw, H, W)
    out = xt.new_zeros(R, oc, ph, pw)
    for i in range(ph):
        hs = torch.floor(i * bh + y1).long().clamp(0, H)
        he = torch.ceil((i + 1) * bh + y1).long().clamp(0, H)
        mh = ((hh[None] >= hs[:, None]) & (hh[None] < he[:, None])).to(xt.dtype)
        for j in range(pw):
            ws = torch.floor(j * bw + x1).long().clamp(0, W)
            we = torch.ceil((j + 1) * bw + x1).long().clamp(0, W)
            mw = ((ww[None] >= ws[:, None]) & (ww[None] < we[:, None])).to(xt.dtype)
            m = mh[:, :, None] * mw[:, None, :]  # [R,H,W]
            area = m.sum(dim=(1, 2))
            s = (feat[:, :, i, j] * m[:, None]).sum(dim=(2, 3))
            out[:, :, i, j] = torch.where(area[:, None] > 0, s / area.clamp(min=1)[:, None],
                                          torch.zeros_like(s))
    return _w(out)


class RoIAlign(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self._output_size, self._spatial_scale,
                         aligned=aligned)


class RoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self._output_size, self._spatial_scale)

    def extra_repr(self):
        return f'output_size={self._output_size}, spatial_scale={self._spatial_scale}'


class PSRoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


# ----------------------------------------------------------------------------
# NMS family
# ----------------------------------------------------------------------------
def _iou_matrix(a, b, normalized=True):
    off = 0.0 if normalized else 1.0
    area_a = (a[:, 2] - a[:, 0] + off).clamp(min=0) * (a[:, 3] - a[:, 1] + off).clamp(min=0)
    area_b = (b[:, 2] - b[:, 0] + off).clamp(min=0) * (b[:, 3] - b[:, 1] + off).clamp(min=0)
    lt = torch.maximum(a[:, None, :2], b[None, :, :2])
    rb = torch.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt + off).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area_a[:, None] + area_b[None, :] - inter).clamp(min=1e-10)


def _greedy_nms(boxes, thresh):
    """Indices (into ``boxes``, already in priority order) kept by greedy NMS."""
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.long, device=boxes.device)
    iou = _iou_matrix(boxes.float(), boxes.float()).cpu()
    keep = torch.ones(n, dtype=torch.bool)
    sup = (iou > thresh)
    for i in range(n):
        if keep[i]:
            s = sup[i].clone()
            s[:i + 1] = False
            keep &= ~s
    return torch.nonzero(keep).flatten().to(boxes.device)


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None,
        top_k=None):
    """Greedy non-maximum suppression; with ``scores`` boxes are visited by descending score,
    with ``category_idxs`` suppression only acts within a category. Returns kept indices
    (int64), sorted by score when scores are given."""
    bt = _u(boxes)
    if scores is None:
        return _w(_greedy_nms(bt, iou_threshold))
    st = _u(scores).reshape(-1)
    if category_idxs is None:
        order = torch.argsort(st, descending=True)
        keep = order[_greedy_nms(bt[order], iou_threshold)]
    else:
        cat = _u(category_idxs).reshape(-1)
        cats = categories if categories is not None else torch.unique(cat).tolist()
        kept = []
        for c in cats:
            idx = torch.nonzero(cat == int(c)).flatten()
            if idx.numel() == 0:
                continue
            order = idx[torch.argsort(st[idx], descending=True)]
            kept.append(order[_greedy_nms(bt[order], iou_threshold)])
        keep = torch.cat(kept) if kept else torch.zeros(0, dtype=torch.long, device=bt.device)
        keep = keep[torch.argsort(st[keep], descending=True)]
    if top_k is not None:
        keep = keep[:top_k]
    return _w(keep)


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k,
               use_gaussian=False, gaussian_sigma=2.0, background_label=0, normalized=True,
               return_index=False, return_rois_num=True, name=None):
    """Matrix NMS (SOLOv2): scores are decayed by the IoU with every higher-scored box of
    the same class instead of hard suppression. bboxes [N,M,4], scores [N,C,M] ->
    out [K,6] rows (label, score, x1, y1, x2, y2), optional index [K,1], rois_num [N]."""
    bt, st = _u(bboxes), _u(scores)
    N, C, M = st.shape
    outs, idxs, nums = [], [], []
    for n in range(N):
        rows, rid = [], []
        for c in range(C):
            if c == background_label:
                continue
            sc = st[n, c]
            cand = torch.nonzero(sc > score_threshold).flatten()
            if cand.numel() == 0:
                continue
            cand = cand[torch.argsort(sc[cand], descending=True)]
            if nms_top_k > -1:
                cand = cand[:nms_top_k]
            b = bt[n, cand].float()
            s = sc[cand].float()
            iou = _iou_matrix(b, b, normalized).triu(diagonal=1)  # iou[i, j], i < j
            max_iou = iou.max(dim=0).values  # per box: max IoU with any higher-scored box
            if use_gaussian:
                decay = torch.exp((max_iou[:, None] ** 2 - iou ** 2) * gaussian_sigma)
            else:
                decay = (1 - iou) / (1 - max_iou[:, None]).clamp(min=1e-10)
            decay = torch.where(torch.ones_like(iou).triu(diagonal=1) > 0, decay,
                                torch.ones_like(decay)).min(dim=0).values
            ds = s * decay
            ok = ds > post_threshold
            for k in torch.nonzero(ok).flatten().tolist():
                rows.append(torch.cat([torch.tensor([float(c), float(ds[k])], device=b.device),
                                       b[k]]))
                rid.append(n * M + int(cand[k]))
        if rows:
            R = torch.stack(rows)
            order = torch.argsort(R[:, 1], descending=True)
            if keep_top_k > -1:
                order = order[:keep_top_k]
            outs.append(R[order])
            idxs.append(torch.tensor(rid, device=R.device)[order])
            nums.append(len(order))
        else:
            nums.append(0)
    out = torch.cat(outs) if outs else torch.zeros(0, 6, device=bt.device)
    res = [_w(out.to(bt.dtype))]
    if return_index:
        idx = torch.cat(idxs) if idxs else torch.zeros(0, dtype=torch.long, device=bt.device)
        res.append(_w(idx.reshape(-1, 1)))
    if return_rois_num:
        res.append(_w(torch.tensor(nums, dtype=torch.int32, device=bt.device)))
    return res[0] if len(res) == 1 else tuple(res)


# ----------------------------------------------------------------------------
# box coding / priors
# ----------------------------------------------------------------------------
def box_coder(prior_box, prior_box_var, target_box, code_type='encode_center_size',
              box_normalized=True, axis=0, name=None):
    """Encode target boxes against priors (center-size deltas) or decode deltas back to
    boxes. encode: target [N,4], prior [M,4] -> [N,M,4]; decode: target [N,M,4] with
    priors broadcast along ``axis``."""
    pb = _u(prior_box)
    tb = _u(target_box)
    off = 0.0 if box_normalized else 1.0
    if prior_box_var is None:
        var = None
    elif isinstance(prior_box_var, (list, tuple)):
        var = torch.tensor(prior_box_var, dtype=pb.dtype, device=pb.device)
    else:
        var = _u(prior_box_var)
    pw = pb[:, 2] - pb[:, 0] + off
    ph = pb[:, 3] - pb[:, 1] + off
    pcx = pb[:, 0] + pw / 2
    pcy = pb[:, 1] + ph / 2
    if code_type.lower() in ('encode_center_size', 'encode'):
        tw = tb[:, 2] - tb[:, 0] + off
        th = tb[:, 3] - tb[:, 1] + off
        tcx = tb[:, 0] + tw / 2
        tcy = tb[:, 1] + th / 2
        out = torch.stack([(tcx[:, None] - pcx[None]) / pw[None],
                           (tcy[:, None] - pcy[None]) / ph[None],
                           torch.log((tw[:, None] / pw[None]).abs()),
                           torch.log((th[:, None] / ph[None]).abs())], dim=-1)
        if var is not None:
            out = out / (var if var.dim() == 1 else var[None])
        return _w(out)
    # decode
    if tb.dim() == 2:
        tb = tb[:, None, :] if axis == 0 else tb[None]
    if axis == 0:
        pw_, ph_, pcx_, pcy_ = pw[None], ph[None], pcx[None], pcy[None]
        v = None if var is None else (var if var.dim() == 1 else var[None])
    else:
        pw_, ph_, pcx_, pcy_ = pw[:, None], ph[:, None], pcx[:, None], pcy[:, None]
        v = None if var is None else (var if var.dim() == 1 else var[:, None])
    d = tb if v is None else tb * v
    cx = d[..., 0] * pw_ + pcx_
    cy = d[..., 1] * ph_ + pcy_
    w = torch.exp(d[..., 2]) * pw_
    h = torch.exp(d[..., 3]) * ph_
    return _w(torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1))


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=(1.0,),
              variance=(0.1, 0.1, 0.2, 0.2), flip=False, clip=False, steps=(0.0, 0.0),
              offset=0.5, min_max_aspect_ratios_order=False, name=None):
    """SSD prior boxes for every feature-map cell -> (boxes, variances), each
    [H, W, num_priors, 4], normalized to the image size."""
    H, W = _u(input).shape[2:]
    IH, IW = _u(image).shape[2:]
    dev = _u(input).device
    ars = [1.0]
    for ar in aspect_ratios:
        for a in ([ar, 1.0 / ar] if flip else [ar]):
            if all(abs(a - e) > 1e-6 for e in ars):
                ars.append(a)
    sw = steps[0] if steps[0] > 0 else IW / W
    sh = steps[1] if steps[1] > 0 else IH / H
    whs = []
    for s, mn in enumerate(min_sizes):
        mx = max_sizes[s] if max_sizes else None
        if min_max_aspect_ratios_order:
            whs.append((mn, mn))
            if mx is not None:
                whs.append((math.sqrt(mn * mx),) * 2)
            for a in ars:
                if abs(a - 1.0) > 1e-6:
                    whs.append((mn * math.sqrt(a), mn / math.sqrt(a)))
        else:
            for a in ars:
                whs.append((mn * math.sqrt(a), mn / math.sqrt(a)))
            if mx is not None:
                whs.append((math.sqrt(mn * mx),) * 2)
    wh = torch.tensor(whs, dtype=torch.float32, device=dev)  # [P,2]
    cx = (torch.arange(W, device=dev, dtype=torch.float32) + offset) * sw
    cy = (torch.arange(H, device=dev, dtype=torch.float32) + offset) * sh
    cxg = cx[None, :, None].expand(H, W, len(whs))
    cyg = cy[:, None, None].expand(H, W, len(whs))
    bw, bh = wh[:, 0][None, None] / 2, wh[:, 1][None, None] / 2
    boxes = torch.stack([(cxg - bw) / IW, (cyg - bh) / IH, (cxg + bw) / IW, (cyg + bh) / IH], -1)
    if clip:
        boxes = boxes.clamp(0.0, 1.0)
    var = torch.tensor(list(variance), dtype=torch.float32, device=dev).expand_as(boxes)
    return _w(boxes.contiguous()), _w(var.contiguous())


# ----------------------------------------------------------------------------
# YOLOv3
# ----------------------------------------------------------------------------
def _yolo_split(xt, na, class_num, iou_aware):
    N, _, H, W = xt.shape
    ious = None
    if iou_aware:
        ious = xt[:, :na]
        xt = xt[:, na:]
    p = xt.reshape(N, na, 5 + class_num, H, W)
    return p, ious


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True,
             name=None, scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    """Decode a YOLOv3 head into image-space boxes [N, A*H*W, 4] and per-class scores
    [N, A*H*W, class_num]; predictions under ``conf_thresh`` are zeroed."""
    xt = _u(x)
    N, _, H, W = xt.shape
    an = torch.tensor(anchors, dtype=xt.dtype, device=xt.device).reshape(-1, 2)
    na = an.shape[0]
    p, ious = _yolo_split(xt, na, class_num, iou_aware)
    ims = _u(img_size).to(xt.dtype)
    img_h, img_w = ims[:, 0][:, None, None, None], ims[:, 1][:, None, None, None]
    gx = torch.arange(W, device=xt.device, dtype=xt.dtype)[None, None, None, :]
    gy = torch.arange(H, device=xt.device, dtype=xt.dtype)[None, None, :, None]
    bias = -0.5 * (scale_x_y - 1.0)
    cx = (gx + torch.sigmoid(p[:, :, 0]) * scale_x_y + bias) * img_w / W
    cy = (gy + torch.sigmoid(p[:, :, 1]) * scale_x_y + bias) * img_h / H
    in_w, in_h = downsample_ratio * W, downsample_ratio * H
    bw = torch.exp(p[:, :, 2]) * an[:, 0][None, :, None, None] * img_w / in_w
    bh = torch.exp(p[:, :, 3]) * an[:, 1][None, :, None, None] * img_h / in_h
    conf = torch.sigmoid(p[:, :, 4])
    if iou_aware:
        conf = conf.pow(1 - iou_aware_factor) * torch.sigmoid(ious).pow(iou_aware_factor)
    keep = (conf >= conf_thresh).to(xt.dtype)
    x1, y1, x2, y2 = cx - bw / 2, cy - bh / 2, cx + bw / 2, cy + bh / 2
    if clip_bbox:
        x1, x2 = x1.clamp(min=0), torch.minimum(x2, img_w - 1)
        y1, y2 = y1.clamp(min=0), torch.minimum(y2, img_h - 1)
    boxes = torch.stack([x1, y1, x2, y2], -1) * keep[..., None]
    scores = torch.sigmoid(p[:, :, 5:]) * (conf * keep)[:, :, None]
    boxes = boxes.reshape(N, na * H * W, 4)
    scores = scores.permute(0, 1, 3, 4, 2).reshape(N, na * H * W, class_num)
    return _w(boxes), _w(scores)


def _box_iou_cxcywh(a, b):
    ax1, ay1, ax2, ay2 = a[..., 0] - a[..., 2] / 2, a[..., 1] - a[..., 3] / 2, \
        a[..., 0] + a[..., 2] / 2, a[..., 1] + a[..., 3] / 2
    bx1, by1, bx2, by2 = b[..., 0] - b[..., 2] / 2, b[..., 1] - b[..., 3] / 2, \
        b[..., 0] + b[..., 2] / 2, b[..., 1] + b[..., 3] / 2
    iw = (torch.minimum(ax2, bx2) - torch.maximum(ax1, bx1)).clamp(min=0)
    ih = (torch.minimum(ay2, by2) - torch.maximum(ay1, by1)).clamp(min=0)
    inter = iw * ih
    return inter / (a[..., 2] * a[..., 3] + b[..., 2] * b[..., 3] - inter).clamp(min=1e-10)


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh,
              downsample_ratio, gt_score=None, use_label_smooth=True, name=None,
              scale_x_y=1.0):
    """YOLOv3 loss per image [N]: every ground truth (normalized cx, cy, w, h) is assigned
    to the anchor of best shape IoU; if that anchor belongs to this head it supervises the
    cell's x/y (sigmoid CE), w/h (L1 on log-space) scaled by (2 - w*h), objectness and
    classes (sigmoid CE, optional label smoothing). Predictions whose best IoU with any
    ground truth exceeds ``ignore_thresh`` are not penalized as background."""
    xt = _u(x)
    gb = _u(gt_box).to(xt.dtype)
    gl = _u(gt_label).long()
    N, _, H, W = xt.shape
    B = gb.shape[1]
    all_an = torch.tensor(anchors, dtype=xt.dtype, device=xt.device).reshape(-1, 2)
    mask = list(anchor_mask)
    na = len(mask)
    an = all_an[mask]
    p = xt.reshape(N, na, 5 + class_num, H, W)
    gs = torch.ones(N, B, dtype=xt.dtype, device=xt.device) if gt_score is None \
        else _u(gt_score).to(xt.dtype)
    in_w, in_h = downsample_ratio * W, downsample_ratio * H
    bias = -0.5 * (scale_x_y - 1.0)
    gxg = torch.arange(W, device=xt.device, dtype=xt.dtype)[None, None, None, :]
    gyg = torch.arange(H, device=xt.device, dtype=xt.dtype)[None, None, :, None]
    # predicted boxes (normalized cx, cy, w, h) for the ignore mask (no gradient)
    with torch.no_grad():
        pcx = (gxg + torch.sigmoid(p[:, :, 0]) * scale_x_y + bias) / W
        pcy = (gyg + torch.sigmoid(p[:, :, 1]) * scale_x_y + bias) / H
        pw_ = torch.exp(p[:, :, 2]) * an[:, 0][None, :, None, None] / in_w
        ph_ = torch.exp(p[:, :, 3]) * an[:, 1][None, :, None, None] / in_h
        pred = torch.stack([pcx, pcy, pw_, ph_], -1).reshape(N, -1, 1, 4)
        valid_gt = (gb[..., 2] > 0) & (gb[..., 3] > 0)
        iou = _box_iou_cxcywh(pred, gb[:, None, :, :])  # [N, na*H*W, B]
        iou = torch.where(valid_gt[:, None, :], iou, torch.zeros_like(iou))
        best = iou.max(dim=2).values.reshape(N, na, H, W)
        noobj = (best <= ignore_thresh).to(xt.dtype)
    obj_t = torch.zeros(N, na, H, W, dtype=xt.dtype, device=xt.device)
    tx = torch.zeros_like(obj_t)
    ty, tw, th, tscale = torch.zeros_like(obj_t), torch.zeros_like(obj_t), \
        torch.zeros_like(obj_t), torch.zeros_like(obj_t)
    tcls = torch.zeros(N, na, class_num, H, W, dtype=xt.dtype, device=xt.device)
    pos = torch.zeros(N, na, H, W, dtype=torch.bool, device=xt.device)
    # best anchor by shape IoU (centered boxes)
    gwh = gb[..., 2:4]
    inter = torch.minimum(gwh[..., None, 0] * in_w, all_an[:, 0]) * \
        torch.minimum(gwh[..., None, 1] * in_h, all_an[:, 1])
    union = gwh[..., None, 0] * in_w * gwh[..., None, 1] * in_h + \
        all_an[:, 0] * all_an[:, 1] - inter
    best_an = (inter / union.clamp(min=1e-10)).argmax(-1)  # [N,B]
    pos_v = 1.0 - 1.0 / class_num if use_label_smooth else 1.0
    neg_v = 1.0 / class_num if use_label_smooth else 0.0
    for n in range(N):
        for t in range(B):
            if gb[n, t, 2] <= 0 or gb[n, t, 3] <= 0:
                continue
            a_all = int(best_an[n, t])
            if a_all not in mask:
                continue
            a = mask.index(a_all)
            gi = min(max(int(gb[n, t, 0] * W), 0), W - 1)
            gj = min(max(int(gb[n, t, 1] * H), 0), H - 1)
            pos[n, a, gj, gi] = True
            sc = gs[n, t]
            obj_t[n, a, gj, gi] = sc
            tx[n, a, gj, gi] = gb[n, t, 0] * W - gi
            ty[n, a, gj, gi] = gb[n, t, 1] * H - gj
            tw[n, a, gj, gi] = torch.log(gb[n, t, 2] * in_w / all_an[a_all, 0])
            th[n, a, gj, gi] = torch.log(gb[n, t, 3] * in_h / all_an[a_all, 1])
            tscale[n, a, gj, gi] = (2.0 - gb[n, t, 2] * gb[n, t, 3]) * sc
            tcls[n, a, :, gj, gi] = neg_v
            tcls[n, a, int(gl[n, t]), gj, gi] = pos_v
    posf = pos.to(xt.dtype)
    bce = TF.binary_cross_entropy_with_logits
    lxy = (bce(p[:, :, 0], tx, reduction='none') + bce(p[:, :, 1], ty, reduction='none')) * \
        tscale * posf
    lwh = ((p[:, :, 2] - tw).abs() + (p[:, :, 3] - th).abs()) * tscale * posf
    lobj_pos = bce(p[:, :, 4], torch.ones_like(obj_t), reduction='none') * obj_t * posf
    lobj_neg = bce(p[:, :, 4], torch.zeros_like(obj_t), reduction='none') * noobj * (1 - posf)
    lcls = (bce(p[:, :, 5:], tcls, reduction='none').sum(2)) * obj_t * posf
    loss = (lxy + lwh + lobj_pos + lobj_neg + lcls).sum(dim=(1, 2, 3))
    return _w(loss)


# ----------------------------------------------------------------------------
# deformable convolution
# ----------------------------------------------------------------------------
def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1,
                  deformable_groups=1, groups=1, mask=None, name=None):
    """Deformable convolution v1 (``mask=None``) / v2: every kernel tap samples the input
    bilinearly at its offset position (times the modulation mask), then one grouped GEMM
    with the weights. offset [N, 2*dg*kh*kw, Ho, Wo] as (dy, dx) pairs per tap."""
    xt, ot, wt = _u(x), _u(offset), _u(weight)
    N, C, H, W = xt.shape
    O, Cg, kh, kw = wt.shape
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    Ho, Wo = ot.shape[2], ot.shape[3]
    K = kh * kw
    dg = deformable_groups
    off = ot.reshape(N, dg, K, 2, Ho, Wo)
    ky = (torch.arange(kh, device=xt.device) * dh).repeat_interleave(kw).to(xt.dtype)
    kx = (torch.arange(kw, device=xt.device) * dw).repeat(kh).to(xt.dtype)
    oy = (torch.arange(Ho, device=xt.device) * sh - ph).to(xt.dtype)
    ox = (torch.arange(Wo, device=xt.device) * sw - pw).to(xt.dtype)
    Y = oy[None, None, None, :, None] + ky[None, None, :, None, None] + off[:, :, :, 0]
    X = ox[None, None, None, None, :] + kx[None, None, :, None, None] + off[:, :, :, 1]
    # [N, dg, K, Ho, Wo] sample positions; channels of group g use offsets of group g
    cpg = C // dg
    xg = xt.reshape(N * dg, cpg, H, W)
    bidx = torch.arange(N * dg, device=xt.device)[:, None, None, None]
    vals = _bilinear_dcn(xg, bidx, Y.reshape(N * dg, K, Ho, Wo), X.reshape(N * dg, K, Ho, Wo))
    # vals [N*dg, K, Ho, Wo, cpg]
    if mask is not None:
        m = _u(mask).reshape(N * dg, K, Ho, Wo)
        vals = vals * m[..., None]
    cols = vals.reshape(N, dg, K, Ho * Wo, cpg).permute(0, 1, 4, 2, 3).reshape(N, C, K, Ho * Wo)
    cols = cols.reshape(N, groups, Cg * K, Ho * Wo)
    wg = wt.reshape(groups, O // groups, Cg * K)
    out = torch.einsum('gok,ngkp->ngop', wg, cols).reshape(N, O, Ho, Wo)
    if bias is not None:
        out = out + _u(bias).reshape(1, -1, 1, 1)
    return _w(out)


class DeformConv2D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0,
                 dilation=1, deformable_groups=1, groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        assert in_channels % groups == 0 and out_channels % groups == 0
        self._in_channels, self._out_channels = in_channels, out_channels
        self._kernel_size = _pair(kernel_size)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._deformable_groups, self._groups = deformable_groups, groups
        from ..nn import initializer as I
        fan_in = in_channels // groups * self._kernel_size[0] * self._kernel_size[1]
        self.weight = self.create_parameter(
            [out_channels, in_channels // groups, *self._kernel_size], attr=weight_attr,
            default_initializer=I.Normal(0.0, (2.0 / fan_in) ** 0.5))
        self.bias = None if bias_attr is False else self.create_parameter(
            [out_channels], attr=bias_attr, is_bias=True)

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self._stride, self._padding,
                             self._dilation, self._deformable_groups, self._groups, mask)


# ----------------------------------------------------------------------------
# proposals
# ----------------------------------------------------------------------------
def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale,
                             pixel_offset=False, rois_num=None, name=None):
    """Assign every RoI to an FPN level by its scale:
    level = floor(log2(sqrt(area) / refer_scale + 1e-8) + refer_level), clipped.
    Returns (multi_rois per level, restore_index [R,1], rois_num per level or None)."""
    rt = _u(fpn_rois)
    off = 1.0 if pixel_offset else 0.0
    w = (rt[:, 2] - rt[:, 0] + off).clamp(min=0)
    h = (rt[:, 3] - rt[:, 1] + off).clamp(min=0)
    lvl = torch.floor(torch.log2(torch.sqrt(w * h) / refer_scale + 1e-8) + refer_level)
    lvl = lvl.clamp(min_level, max_level).long()
    R = rt.shape[0]
    img = _batch_index(rois_num, R, rt.device)
    multi, order, nums = [], [], []
    n_img = int(_u(rois_num).numel()) if rois_num is not None else 1
    for L in range(min_level, max_level + 1):
        idx = torch.nonzero(lvl == L).flatten()
        idx = idx[torch.argsort(img[idx] * (R + 1) + idx)]  # keep image-major order
        multi.append(_w(rt[idx]))
        order.append(idx)
        if rois_num is not None:
            nums.append(_w(torch.bincount(img[idx], minlength=n_img).to(torch.int32)))
    cat = torch.cat(order)
    restore = torch.empty_like(cat)
    restore[cat] = torch.arange(cat.numel(), device=cat.device)
    return multi, _w(restore.reshape(-1, 1)), (nums if rois_num is not None else None)


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000,
                       post_nms_top_n=1000, nms_thresh=0.5, min_size=0.1, eta=1.0,
                       pixel_offset=False, return_rois_num=False, name=None):
    """RPN proposals per image: top ``pre_nms_top_n`` anchors by score, decode deltas
    (with variances), clip to the image, drop boxes smaller than ``min_size``, NMS, keep
    ``post_nms_top_n``. Returns (rois [R,4], probs [R,1][, rois_num [N]])."""
    st, dt = _u(scores), _u(bbox_deltas)
    ims = _u(img_size)
    an = _u(anchors).reshape(-1, 4)
    va = _u(variances).reshape(-1, 4)
    N, A, H, W = st.shape
    off = 1.0 if pixel_offset else 0.0
    rois, probs, nums = [], [], []
    for n in range(N):
        s = st[n].permute(1, 2, 0).reshape(-1)
        d = dt[n].reshape(A, 4, H, W).permute(2, 3, 0, 1).reshape(-1, 4)
        k = min(pre_nms_top_n, s.numel()) if pre_nms_top_n > 0 else s.numel()
        top = torch.topk(s, k).indices
        s, d, a, v = s[top], d[top], an[top], va[top]
        aw = a[:, 2] - a[:, 0] + off
        ah = a[:, 3] - a[:, 1] + off
        acx, acy = a[:, 0] + 0.5 * aw, a[:, 1] + 0.5 * ah
        cx = v[:, 0] * d[:, 0] * aw + acx
        cy = v[:, 1] * d[:, 1] * ah + acy
        w = torch.exp(torch.clamp(v[:, 2] * d[:, 2], max=math.log(1000.0 / 16))) * aw
        h = torch.exp(torch.clamp(v[:, 3] * d[:, 3], max=math.log(1000.0 / 16))) * ah
        b = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2 - off, cy + h / 2 - off], -1)
        ih, iw = float(ims[n, 0]), float(ims[n, 1])
        b = torch.stack([b[:, 0].clamp(0, iw - off), b[:, 1].clamp(0, ih - off),
                         b[:, 2].clamp(0, iw - off), b[:, 3].clamp(0, ih - off)], -1)
        bw = b[:, 2] - b[:, 0] + off
        bh = b[:, 3] - b[:, 1] + off
        ok = (bw >= max(min_size, 1.0 if pixel_offset else 0.0)) & \
            (bh >= max(min_size, 1.0 if pixel_offset else 0.0))
        b, s = b[ok], s[ok]
        keep = _greedy_nms(b, nms_thresh)[:post_nms_top_n]
        rois.append(b[keep])
        probs.append(s[keep].reshape(-1, 1))
        nums.append(int(keep.numel()))
    out = (_w(torch.cat(rois)), _w(torch.cat(probs)))
    if return_rois_num:
        out = out + (_w(torch.tensor(nums, dtype=torch.int32, device=st.device)),)
    return out


# ----------------------------------------------------------------------------
# image IO
# ----------------------------------------------------------------------------
def read_file(filename, name=None):
    """Raw bytes of a file as a 1-D uint8 tensor."""
    with open(filename, 'rb') as f:
        data = f.read()
    return _w(torch.frombuffer(bytearray(data), dtype=torch.uint8).clone())


def decode_jpeg(x, mode='unchanged', name=None):
    """Decode JPEG bytes (1-D uint8 tensor) to a CHW uint8 tensor ('unchanged' | 'gray' |
    'rgb')."""
    import io as _io
    from PIL import Image
    raw = bytes(_u(x).cpu().numpy().tobytes())
    img = Image.open(_io.BytesIO(raw))
    if mode == 'gray':
        img = img.convert('L')
    elif mode == 'rgb':
        img = img.convert('RGB')
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[None]
    else:
        arr = arr.transpose(2, 0, 1)
    return _w(torch.from_numpy(np.array(arr, copy=True)).to(_u(x).device))


class ConvNormActivation(Sequential):
    """Conv2D -> norm layer -> activation block (padding defaults to 'same' for odd k)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=None,
                 groups=1, norm_layer=BatchNorm2D, activation_layer=ReLU, dilation=1,
                 bias=None):
        if padding is None:
            padding = (kernel_size - 1) // 2 * dilation
        if bias is None:
            bias = norm_layer is None
        layers = [Conv2D(in_channels, out_channels, kernel_size, stride, padding,
                         dilation=dilation, groups=groups, bias_attr=None if bias else False)]
        if norm_layer is not None:
            layers.append(norm_layer(out_channels))
        if activation_layer is not None:
            layers.append(activation_layer())
        super().__init__(*layers)
