"""paddle.vision.transforms.functional (parity: python/paddle/vision/transforms/
functional.py with its PIL / cv2-numpy / tensor backends).

One implementation on CHW float tensors (torch): numpy HWC arrays and PIL images are
converted in, transformed, and converted back to their own kind and dtype (uint8 results
are rounded and clamped). Geometric warps (rotate / affine / perspective) use an inverse
sampling grid; color ops blend with a degenerate image as in the reference.
"""
import math
import numbers

import numpy as np
import torch
import torch.nn.functional as TF

from ...framework.core import Tensor, _u

_INTERP = {'nearest': 'nearest', 'bilinear': 'bilinear', 'bicubic': 'bicubic',
           'linear': 'bilinear', 'area': 'area', 'lanczos': 'bicubic'}


def _is_pil(img):
    try:
        from PIL import Image
        return isinstance(img, Image.Image)
    except ImportError:  # pragma: no cover
        return False


def _to_chw(img, data_format='CHW'):
    """-> (float32 CHW torch tensor, restore fn)."""
    if isinstance(img, Tensor) or torch.is_tensor(img):
        t = _u(img)
        dt = t.dtype
        squeeze = t.dim() == 2
        t = t[None] if squeeze else t
        hwc = data_format == 'HWC'
        if hwc:
            t = t.permute(2, 0, 1)

        def back(o):
            o = o.permute(1, 2, 0) if hwc else o
            o = o[0] if squeeze else o
            if dt == torch.uint8:
                o = o.round().clamp(0, 255)
            return Tensor(o.to(dt))
        return t.float(), back
    if _is_pil(img):
        from PIL import Image
        mode = img.mode
        a = np.asarray(img)

        def back(o):
            arr = o.round().clamp(0, 255).to(torch.uint8).permute(1, 2, 0).cpu().numpy()
            if arr.shape[2] == 1:
                arr = arr[:, :, 0]
            return Image.fromarray(arr, mode=mode if mode in ('L', 'RGB', 'RGBA') else None)
    else:
        a = np.asarray(img)
        dt = a.dtype

        def back(o):
            arr = o.permute(1, 2, 0).cpu().numpy()
            if a.ndim == 2:
                arr = arr[:, :, 0]
            if dt == np.uint8:
                arr = np.clip(np.round(arr), 0, 255)
            return arr.astype(dt)
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).permute(2, 0, 1), back


def _size_hw(img):
    if _is_pil(img):
        return img.size[1], img.size[0]
    if isinstance(img, Tensor) or torch.is_tensor(img):
        s = _u(img).shape
        return (s[-2], s[-1])
    s = np.asarray(img).shape
    return s[0], s[1]


def _max_val(img):
    if isinstance(img, Tensor) or torch.is_tensor(img):
        return 255.0 if _u(img).dtype == torch.uint8 else 1.0
    if _is_pil(img):
        return 255.0
    return 255.0 if np.asarray(img).dtype == np.uint8 else 1.0


# ----------------------------------------------------------------------------
# conversion
# ----------------------------------------------------------------------------
def to_tensor(pic, data_format='CHW'):
    """HWC uint8/float image -> float32 Tensor (uint8 scaled to [0, 1])."""
    if isinstance(pic, Tensor):
        return pic
    a = np.asarray(pic)
    if a.ndim == 2:
        a = a[:, :, None]
    scale = a.dtype == np.uint8
    a = a.astype(np.float32)
    if scale:
        a = a / 255.0
    if data_format == 'CHW':
        a = a.transpose(2, 0, 1)
    return Tensor(torch.from_numpy(np.ascontiguousarray(a)))


def normalize(img, mean, std, data_format='CHW', to_rgb=False):
    if isinstance(img, Tensor):
        t = _u(img).float()
        shp = (-1, 1, 1) if data_format == 'CHW' else (1, 1, -1)
        if to_rgb:
            t = t.flip(0) if data_format == 'CHW' else t.flip(-1)
        m = torch.as_tensor(np.asarray(mean, np.float32)).reshape(shp)
        s = torch.as_tensor(np.asarray(std, np.float32)).reshape(shp)
        return Tensor((t - m) / s)
    a = np.asarray(img).astype(np.float32)
    if to_rgb:
        a = a[::-1] if data_format == 'CHW' else a[..., ::-1]
    shp = (-1, 1, 1) if data_format == 'CHW' else (1, 1, -1)
    return (a - np.asarray(mean, np.float32).reshape(shp)) / \
        np.asarray(std, np.float32).reshape(shp)


# ----------------------------------------------------------------------------
# geometry
# ----------------------------------------------------------------------------
def resize(img, size, interpolation='bilinear'):
    """``size`` int: shorter side -> size keeping aspect; (h, w): exact."""
    h, w = _size_hw(img)
    if isinstance(size, numbers.Number):
        if (w <= h and w == size) or (h <= w and h == size):
            return img
        if w < h:
            ow, oh = int(size), int(size * h / w)
        else:
            oh, ow = int(size), int(size * w / h)
    else:
        oh, ow = int(size[0]), int(size[1])
    t, back = _to_chw(img)
    mode = _INTERP.get(interpolation, 'bilinear')
    kw = {} if mode in ('nearest', 'area') else {'align_corners': False}
    o = TF.interpolate(t[None], size=(oh, ow), mode=mode, **kw)[0]
    return back(o)


def crop(img, top, left, height, width):
    t, back = _to_chw(img)
    return back(t[:, top:top + height, left:left + width])


def center_crop(img, output_size):
    th, tw = (output_size, output_size) if isinstance(output_size, numbers.Number) \
        else output_size
    h, w = _size_hw(img)
    return crop(img, int(round((h - th) / 2.0)), int(round((w - tw) / 2.0)), th, tw)


def hflip(img):
    t, back = _to_chw(img)
    return back(t.flip(-1))


def vflip(img):
    t, back = _to_chw(img)
    return back(t.flip(-2))


def pad(img, padding, fill=0, padding_mode='constant'):
    """padding: int | (lr, tb) | (l, t, r, b); modes constant | edge | reflect | symmetric."""
    if isinstance(padding, numbers.Number):
        l = t_ = r = b = int(padding)
    elif len(padding) == 2:
        l = r = int(padding[0])
        t_ = b = int(padding[1])
    else:
        l, t_, r, b = (int(p) for p in padding)
    t, back = _to_chw(img)
    if padding_mode == 'constant':
        if isinstance(fill, (tuple, list)):
            out = torch.empty(t.shape[0], t.shape[1] + t_ + b, t.shape[2] + l + r)
            for c in range(t.shape[0]):
                out[c] = fill[c % len(fill)]
            out[:, t_:t_ + t.shape[1], l:l + t.shape[2]] = t
        else:
            out = TF.pad(t, (l, r, t_, b), value=float(fill))
    elif padding_mode == 'edge':
        out = TF.pad(t[None], (l, r, t_, b), mode='replicate')[0]
    elif padding_mode == 'reflect':
        out = TF.pad(t[None], (l, r, t_, b), mode='reflect')[0]
    elif padding_mode == 'symmetric':
        out = torch.from_numpy(np.pad(t.numpy(), ((0, 0), (t_, b), (l, r)), mode='symmetric'))
    else:
        raise ValueError(f"unsupported padding_mode {padding_mode}")
    return back(out)


def _warp(img, inv, out_hw, interpolation, fill):
    """Sample ``img`` at inv @ [x, y, 1] for every output pixel (pixel-center coords)."""
    t, back = _to_chw(img)
    C, H, W = t.shape
    oh, ow = out_hw
    ys, xs = torch.meshgrid(torch.arange(oh, dtype=torch.float64) + 0.5,
                            torch.arange(ow, dtype=torch.float64) + 0.5, indexing='ij')
    pts = torch.stack([xs, ys, torch.ones_like(xs)], -1) @ torch.as_tensor(inv).T
    if pts.shape[-1] == 3:
        pts = pts[..., :2] / pts[..., 2:3]
    gx = pts[..., 0] / W * 2 - 1
    gy = pts[..., 1] / H * 2 - 1
    grid = torch.stack([gx, gy], -1).float()[None]
    mode = 'nearest' if interpolation == 'nearest' else 'bilinear'
    ones = torch.ones(1, 1, H, W)
    src = torch.cat([t[None], ones], 1)
    o = TF.grid_sample(src, grid, mode=mode, padding_mode='zeros', align_corners=False)[0]
    mask = o[-1:] > 0.5 if mode == 'nearest' else o[-1:]
    val, m = o[:-1], mask.float()
    fillv = torch.as_tensor(fill if isinstance(fill, (tuple, list)) else [fill] * C,
                            dtype=torch.float32).reshape(-1, 1, 1)[:C]
    # val is already coverage-weighted (zero padding): add the fill for the uncovered part
    return back(val + fillv * (1 - m))


def _affine_inv(center, angle, translate, scale, shear):
    """Inverse of T(center+translate) R(angle) Sh(shear) S(scale) T(-center) (3x3)."""
    cx, cy = center
    a = math.radians(angle)
    sx, sy = (math.radians(s) for s in shear)
    # forward matrix (image coords, y down; positive angle = counter-clockwise on screen)
    R = np.array([[math.cos(a), math.sin(a), 0], [-math.sin(a), math.cos(a), 0], [0, 0, 1]])
    Sh = np.array([[1, -math.tan(sx), 0], [-math.tan(sy), 1, 0], [0, 0, 1]])
    S = np.diag([scale, scale, 1.0])
    T1 = np.array([[1, 0, cx + translate[0]], [0, 1, cy + translate[1]], [0, 0, 1]])
    T0 = np.array([[1, 0, -cx], [0, 1, -cy], [0, 0, 1]])
    M = T1 @ R @ Sh @ S @ T0
    return np.linalg.inv(M)


def affine(img, angle, translate, scale, shear, interpolation='nearest', fill=0, center=None):
    h, w = _size_hw(img)
    if isinstance(shear, numbers.Number):
        shear = (shear, 0.0)
    c = center if center is not None else (w * 0.5, h * 0.5)
    return _warp(img, _affine_inv(c, angle, translate, scale, shear), (h, w), interpolation,
                 fill)


def rotate(img, angle, interpolation='nearest', expand=False, center=None, fill=0):
    h, w = _size_hw(img)
    c = center if center is not None else (w * 0.5, h * 0.5)
    inv = _affine_inv(c, angle, (0, 0), 1.0, (0.0, 0.0))
    oh, ow = h, w
    if expand:
        M = np.linalg.inv(inv)
        corners = np.array([[0, 0, 1], [w, 0, 1], [0, h, 1], [w, h, 1]], np.float64) @ M.T
        minx, maxx = corners[:, 0].min(), corners[:, 0].max()
        miny, maxy = corners[:, 1].min(), corners[:, 1].max()
        ow, oh = int(math.ceil(maxx - minx - 1e-6)), int(math.ceil(maxy - miny - 1e-6))
        shift = np.array([[1, 0, minx], [0, 1, miny], [0, 0, 1]])
        inv = inv @ shift
    return _warp(img, inv, (oh, ow), interpolation, fill)


def _perspective_coeffs(startpoints, endpoints):
    """Homography mapping endpoints -> startpoints (output pixel -> input pixel)."""
    A, bvec = [], []
    for (sx, sy), (ex, ey) in zip(startpoints, endpoints):
        A.append([ex, ey, 1, 0, 0, 0, -sx * ex, -sx * ey])
        A.append([0, 0, 0, ex, ey, 1, -sy * ex, -sy * ey])
        bvec += [sx, sy]
    c = np.linalg.lstsq(np.array(A, np.float64), np.array(bvec, np.float64), rcond=None)[0]
    return np.array([[c[0], c[1], c[2]], [c[3], c[4], c[5]], [c[6], c[7], 1.0]])


def perspective(img, startpoints, endpoints, interpolation='nearest', fill=0):
    h, w = _size_hw(img)
    return _warp(img, _perspective_coeffs(startpoints, endpoints), (h, w), interpolation, fill)


# ----------------------------------------------------------------------------
# color
# ----------------------------------------------------------------------------
def _gray(t):
    if t.shape[0] == 1:
        return t
    return (0.299 * t[0] + 0.587 * t[1] + 0.114 * t[2])[None]


def _blend(a, b, ratio, maxv):
    return (ratio * a + (1 - ratio) * b).clamp(0, maxv)


def to_grayscale(img, num_output_channels=1):
    t, back = _to_chw(img)
    g = _gray(t)
    if _is_pil(img):
        from PIL import Image
        arr = g[0].round().clamp(0, 255).to(torch.uint8).numpy()
        out = Image.fromarray(arr, mode='L')
        return out if num_output_channels == 1 else out.convert('RGB')
    return back(g.expand(num_output_channels, -1, -1).contiguous())


def adjust_brightness(img, brightness_factor):
    t, back = _to_chw(img)
    return back(_blend(t, torch.zeros_like(t), brightness_factor, _max_val(img)))


def adjust_contrast(img, contrast_factor):
    t, back = _to_chw(img)
    m = _gray(t).mean()
    return back(_blend(t, torch.full_like(t, float(m)), contrast_factor, _max_val(img)))


def adjust_saturation(img, saturation_factor):
    t, back = _to_chw(img)
    return back(_blend(t, _gray(t).expand_as(t), saturation_factor, _max_val(img)))


def _rgb_to_hsv(t):
    r, g, b = t[0], t[1], t[2]
    maxc, minc = t.max(0).values, t.min(0).values
    v = maxc
    delta = maxc - minc
    s = torch.where(maxc > 0, delta / maxc.clamp(min=1e-12), torch.zeros_like(maxc))
    dc = delta.clamp(min=1e-12)
    rc, gc, bc = (maxc - r) / dc, (maxc - g) / dc, (maxc - b) / dc
    h = torch.where(maxc == r, bc - gc, torch.where(maxc == g, 2.0 + rc - bc, 4.0 + gc - rc))
    h = torch.where(delta > 0, (h / 6.0) % 1.0, torch.zeros_like(h))
    return h, s, v


def _hsv_to_rgb(h, s, v):
    i = torch.floor(h * 6.0)
    f = h * 6.0 - i
    p, q, t_ = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    i = i.long() % 6
    r = torch.stack([v, q, p, p, t_, v])
    g = torch.stack([t_, v, v, q, p, p])
    b = torch.stack([p, p, t_, v, v, q])
    idx = i[None]
    return torch.stack([r.gather(0, idx)[0], g.gather(0, idx)[0], b.gather(0, idx)[0]])


def adjust_hue(img, hue_factor):
    if not -0.5 <= hue_factor <= 0.5:
        raise ValueError("hue_factor must be in [-0.5, 0.5]")
    t, back = _to_chw(img)
    if t.shape[0] == 1:
        return back(t)
    maxv = _max_val(img)
    h, s, v = _rgb_to_hsv(t[:3] / maxv)
    h = (h + hue_factor) % 1.0
    rgb = _hsv_to_rgb(h, s, v) * maxv
    return back(torch.cat([rgb, t[3:]], 0) if t.shape[0] > 3 else rgb)


def erase(img, i, j, h, w, v, inplace=False):
    """Set the (i, j, h, w) box of a CHW Tensor (or HWC array) to ``v``."""
    if isinstance(img, Tensor):
        t = _u(img) if inplace else _u(img).clone()
        t[..., i:i + h, j:j + w] = _u(v) if isinstance(v, Tensor) else torch.as_tensor(v)
        return img if inplace else Tensor(t)
    a = np.asarray(img) if inplace else np.array(img, copy=True)
    a[i:i + h, j:j + w] = v
    return a
