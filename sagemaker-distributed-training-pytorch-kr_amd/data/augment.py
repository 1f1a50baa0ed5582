"""Batched on-device image augmentations for the Oxford-Pet recipe.

The reference trains with an albumentations pipeline executed per image on the CPU by two
DataLoader workers (/root/reference/2_training_oxford-pet_ddp/pytorch_oxford_ddp.py:140-160):

    RandomResizedCrop, GaussNoise(p=.2), VerticalFlip(p=.5),
    OneOf([MotionBlur(p=.2), MedianBlur(3, p=.1), Blur(3, p=.1)], p=.2),
    OneOf([CLAHE(clip_limit=2), Sharpen(), Emboss(), RandomBrightnessContrast()], p=.3),
    HueSaturationValue(p=.3), Normalize(ImageNet)

Here every op works on a whole uint8-decoded batch [N, 3, H, W] (float in [0, 1]) on the GPU; a
per-sample mask selects which images an op applies to, and per-sample parameters (kernel angles,
strengths, hue shifts) are drawn as tensors, so one launch sequence serves the batch and the
host never touches pixels. ``OneOf`` picks one child per sample with the children's probabilities
as weights (albumentations' rule) and applies it with the block's probability.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

from ..ops import _ext


def _u(n, lo, hi, dev, gen):
    return torch.empty(n, device=dev).uniform_(lo, hi, generator=gen)


def _depthwise(x: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    """Per-sample depthwise conv: x [N, C, H, W], k [N, kh, kw] (same kernel for every channel),
    reflect padding. GPU: the HIP kernel of csrc/kernels/augment.hip (as a torch grouped conv with
    N * C groups MIOpen ran its naive fp32 kernel, 5.8 ms of a ResNet-50 step); CPU: one grouped conv."""
    if _ext.use_kernels(x) and x.dtype == torch.float32 and k.shape[-1] == k.shape[-2] and k.shape[-1] in (3, 5, 7):
        return _ext.ext().aug_depthwise(x, k.float())
    n, c, h, w = x.shape
    kh, kw = k.shape[-2:]
    xp = F.pad(x, (kw // 2, kw // 2, kh // 2, kh // 2), mode="reflect")
    wgt = k[:, None].expand(n, c, kh, kw).reshape(n * c, 1, kh, kw)
    y = F.conv2d(xp.reshape(1, n * c, h + kh - 1, w + kw - 1), wgt.to(x.dtype), groups=n * c)
    return y.view(n, c, h, w)


# ------------------------------------------------------------------------------ blurs
def box_blur(x, size: int = 3):
    n = x.shape[0]
    k = torch.full((n, size, size), 1.0 / (size * size), device=x.device)
    return _depthwise(x, k)


def motion_blur(x, gen: Optional[torch.Generator] = None, size: int = 7):
    """Line kernel through the centre at a random angle per sample (albumentations MotionBlur)."""
    n, dev = x.shape[0], x.device
    ang = _u(n, 0.0, math.pi, dev, gen)
    r = (size - 1) / 2
    ys, xs = torch.meshgrid(torch.arange(size, device=dev) - r, torch.arange(size, device=dev) - r, indexing="ij")
    # distance of each kernel cell from the line at angle `ang` through the centre, soft-rasterised
    d = (xs[None] * torch.sin(ang)[:, None, None] - ys[None] * torch.cos(ang)[:, None, None]).abs()
    k = (1.0 - d).clamp(min=0.0)
    k = k / k.sum(dim=(1, 2), keepdim=True)
    return _depthwise(x, k)


def median_blur(x, size: int = 3):
    """size x size median per channel (reflect padding); 3 x 3 on the GPU: a 19-exchange selection
    network per pixel (csrc/kernels/augment.hip)."""
    if size == 3 and _ext.use_kernels(x) and x.dtype == torch.float32:
        return _ext.ext().aug_median3(x)
    n, c, h, w = x.shape
    p = size // 2
    patches = F.unfold(F.pad(x, (p, p, p, p), mode="reflect"), size)   # [N, C*size*size, H*W]
    return patches.view(n, c, size * size, h * w).median(dim=2).values.view(n, c, h, w)


# ------------------------------------------------------------------------------ kernels
def sharpen(x, gen: Optional[torch.Generator] = None, alpha=(0.2, 0.5), lightness=(0.5, 1.0)):
    """Blend of identity and a Laplacian sharpening kernel (albumentations Sharpen)."""
    n, dev = x.shape[0], x.device
    a = _u(n, *alpha, dev, gen)[:, None, None]
    lt = _u(n, *lightness, dev, gen)[:, None, None]
    ident = torch.zeros(n, 3, 3, device=dev)
    ident[:, 1, 1] = 1
    sh = -torch.ones(n, 3, 3, device=dev)
    sh[:, 1, 1:2] = 8 + lt[:, 0]
    return _depthwise(x, (1 - a) * ident + a * sh).clamp_(0, 1)


def emboss(x, gen: Optional[torch.Generator] = None, alpha=(0.2, 0.5), strength=(0.2, 0.7)):
    """Blend of identity and a directional emboss kernel (albumentations Emboss)."""
    n, dev = x.shape[0], x.device
    a = _u(n, *alpha, dev, gen)[:, None, None]
    s = _u(n, *strength, dev, gen)
    em = torch.zeros(n, 3, 3, device=dev)
    em[:, 0, 0] = -1 - s
    em[:, 0, 1] = -s
    em[:, 1, 0] = -s
    em[:, 1, 1] = 1
    em[:, 1, 2] = s
    em[:, 2, 1] = s
    em[:, 2, 2] = 1 + s
    ident = torch.zeros(n, 3, 3, device=dev)
    ident[:, 1, 1] = 1
    return _depthwise(x, (1 - a) * ident + a * em).clamp_(0, 1)


# ------------------------------------------------------------------------------ CLAHE
def clahe(x, clip_limit: float = 2.0, grid: int = 8, bins: int = 256):
    """Contrast-limited adaptive histogram equalisation of the luma channel: per-tile 256-bin
    histograms (one bincount for the whole batch), clipped at clip_limit x the mean bin height
    with the excess spread uniformly, CDF look-up tables, bilinear interpolation between the
    four surrounding tile LUTs per pixel; chroma is kept by shifting RGB by the luma change."""
    n, _, h, w = x.shape
    dev = x.device
    luma = (0.299 * x[:, 0] + 0.587 * x[:, 1] + 0.114 * x[:, 2]).clamp(0, 1)      # [N, H, W]
    q = (luma * (bins - 1)).round().long()
    ty = (torch.arange(h, device=dev) * grid // h).view(1, h, 1)
    tx = (torch.arange(w, device=dev) * grid // w).view(1, 1, w)
    tile = (torch.arange(n, device=dev).view(n, 1, 1) * grid + ty) * grid + tx       # [N, H, W]
    hist = torch.bincount((tile * bins + q).view(-1), minlength=n * grid * grid * bins).float()
    hist = hist.view(n * grid * grid, bins)
    per_tile = hist.sum(dim=1, keepdim=True)
    limit = (clip_limit * per_tile / bins).clamp(min=1.0)
    excess = (hist - limit).clamp(min=0).sum(dim=1, keepdim=True)
    hist = hist.clamp(max=limit) + excess / bins
    cdf = hist.cumsum(dim=1)
    lut = ((cdf - cdf[:, :1]) / (per_tile - cdf[:, :1]).clamp(min=1.0)).clamp(0, 1)
    lut = lut.view(n, grid, grid, bins)
    # bilinear interpolation between tile centres
    fy = ((torch.arange(h, device=dev, dtype=torch.float32) + 0.5) * grid / h - 0.5).clamp(0, grid - 1)
    fx = ((torch.arange(w, device=dev, dtype=torch.float32) + 0.5) * grid / w - 0.5).clamp(0, grid - 1)
    y0 = fy.floor().long()
    x0 = fx.floor().long()
    y1 = (y0 + 1).clamp(max=grid - 1)
    x1 = (x0 + 1).clamp(max=grid - 1)
    wy = (fy - y0.float()).view(1, h, 1)
    wx = (fx - x0.float()).view(1, 1, w)
    bidx = torch.arange(n, device=dev).view(n, 1, 1)

    def at(yy, xx):
        return lut[bidx, yy.view(1, h, 1), xx.view(1, 1, w), q]

    new = ((1 - wy) * ((1 - wx) * at(y0, x0) + wx * at(y0, x1))
           + wy * ((1 - wx) * at(y1, x0) + wx * at(y1, x1)))
    return (x + (new - luma)[:, None]).clamp_(0, 1)


# ------------------------------------------------------------------------------ colour
def rgb_to_hsv(x):
    r, g, b = x[:, 0], x[:, 1], x[:, 2]
    mx, _ = x.max(dim=1)
    mn, _ = x.min(dim=1)
    d = mx - mn
    dz = d.clamp(min=1e-12)
    h = torch.where(mx == r, ((g - b) / dz) % 6, torch.where(mx == g, (b - r) / dz + 2, (r - g) / dz + 4))
    h = torch.where(d > 0, h / 6.0, torch.zeros_like(h))
    s = torch.where(mx > 0, d / mx.clamp(min=1e-12), torch.zeros_like(mx))
    return torch.stack([h, s, mx], dim=1)


def hsv_to_rgb(hsv):
    h, s, v = hsv[:, 0] % 1.0, hsv[:, 1], hsv[:, 2]
    k = torch.stack([(5 + h * 6) % 6, (3 + h * 6) % 6, (1 + h * 6) % 6], dim=1)
    return v[:, None] - v[:, None] * s[:, None] * torch.clamp(torch.minimum(k, 4 - k), 0, 1)


def hue_saturation_value(x, gen: Optional[torch.Generator] = None, hue=20, sat=30, val=20):
    """Per-sample shifts in OpenCV uint8 units (albumentations defaults): hue +-20 of 180,
    saturation and value +-30 / +-20 of 255."""
    n, dev = x.shape[0], x.device
    hsv = rgb_to_hsv(x)
    dh = _u(n, -hue, hue, dev, gen) / 180.0
    ds = _u(n, -sat, sat, dev, gen) / 255.0
    dv = _u(n, -val, val, dev, gen) / 255.0
    hsv = torch.stack([hsv[:, 0] + dh[:, None, None], (hsv[:, 1] + ds[:, None, None]).clamp(0, 1),
                       (hsv[:, 2] + dv[:, None, None]).clamp(0, 1)], dim=1)
    return hsv_to_rgb(hsv)


def brightness_contrast(x, gen: Optional[torch.Generator] = None, brightness=0.2, contrast=0.2):
    n, dev = x.shape[0], x.device
    b = _u(n, -brightness, brightness, dev, gen).view(n, 1, 1, 1)
    c = 1 + _u(n, -contrast, contrast, dev, gen).view(n, 1, 1, 1)
    mu = x.mean(dim=(1, 2, 3), keepdim=True)
    return ((x - mu) * c + mu + b).clamp_(0, 1)


def gauss_noise(x, gen: Optional[torch.Generator] = None, var_limit=(10.0, 50.0)):
    """Additive N(0, var) noise with var drawn per sample in uint8 units (albumentations)."""
    n, dev = x.shape[0], x.device
    std = _u(n, *var_limit, dev, gen).sqrt().view(n, 1, 1, 1) / 255.0
    return (x + torch.randn(x.shape, device=dev, generator=gen) * std).clamp_(0, 1)


# ------------------------------------------------------------------------------ selection
def apply_masked(x, mask, fn):
    """fn on the samples where ``mask`` (bool [N]) holds; the rest pass through."""
    if not bool(mask.any()):
        return x
    idx = mask.nonzero(as_tuple=True)[0]
    out = x.clone()
    out[idx] = fn(x[idx])
    return out


def one_of(x, p, choices, gen: Optional[torch.Generator] = None):
    """albumentations OneOf: with probability p a sample gets exactly one of ``choices`` =
    [(weight, fn)], picked with probabilities proportional to the weights."""
    n, dev = x.shape[0], x.device
    apply = torch.rand(n, device=dev, generator=gen) < p
    w = torch.tensor([c[0] for c in choices], device=dev, dtype=torch.float32)
    pick = torch.multinomial((w / w.sum()).expand(n, -1), 1, generator=gen).view(n)
    for i, (_, fn) in enumerate(choices):
        x = apply_masked(x, apply & (pick == i), fn)
    return x
