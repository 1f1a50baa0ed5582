"""Swin Transformer (v1) — the model the reference's Oxford-Pet run actually trains
(`model_name: swin_b`, NB2:445-459). torchvision is not available in this
image, so the architecture is implemented here with torchvision's parameter names
(``features.{i}...``, ``norm``, ``head``) so state dicts interchange with ``torchvision.models``.

MI355X layout choices: activations stay channels-last [B, H, W, C] end to end (the natural Swin
layout; no NCHW<->NHWC permutes between blocks), LayerNorms run on the fused HIP LN kernel, window
attention (49 tokens) is a batched bf16 GEMM pair on hipBLASLt with the additive relative-position
bias + shift mask folded into one precomputed [nW, heads, 49, 49] bias per stage.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import functional as SF

CONFIGS = {
    "swin_t": dict(embed_dim=96, depths=[2, 2, 6, 2], num_heads=[3, 6, 12, 24], stochastic_depth_prob=0.2),
    "swin_s": dict(embed_dim=96, depths=[2, 2, 18, 2], num_heads=[3, 6, 12, 24], stochastic_depth_prob=0.3),
    "swin_b": dict(embed_dim=128, depths=[2, 2, 18, 2], num_heads=[4, 8, 16, 32], stochastic_depth_prob=0.5),
}


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose forward runs the fused HIP kernel on GPU (same params / state dict)."""

    def forward(self, x):
        if x.is_cuda and x.shape[-1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float16, torch.float32) \
                and self.weight.dtype in (x.dtype, torch.float32):  # fp32 params under bf16 autocast
            shp = x.shape
            y = SF.layer_norm(x.reshape(-1, shp[-1]), self.weight, self.bias, self.eps)
            return y.view(shp)
        return F.layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)


def _stochastic_depth(x, p: float, training: bool):
    if not training or p == 0.0:
        return x
    keep = 1.0 - p
    mask = torch.empty((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype, device=x.device).bernoulli_(keep)
    return x * mask / keep


def _rel_index(ws: int) -> torch.Tensor:
    c = torch.stack(torch.meshgrid(torch.arange(ws), torch.arange(ws), indexing="ij")).flatten(1)  # [2, N]
    r = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0)                                            # [N, N, 2]
    r[..., 0] += ws - 1
    r[..., 1] += ws - 1
    r[..., 0] *= 2 * ws - 1
    return r.sum(-1).flatten()


class ShiftedWindowAttention(nn.Module):
    def __init__(self, dim: int, window: int, shift: int, num_heads: int, attention_dropout=0.0, dropout=0.0):
        super().__init__()
        self.window, self.shift, self.num_heads = window, shift, num_heads
        self.attention_dropout, self.dropout = attention_dropout, dropout
        self.qkv = nn.Linear(dim, dim * 3)
        self.proj = nn.Linear(dim, dim)
        self.relative_position_bias_table = nn.Parameter(torch.zeros((2 * window - 1) ** 2, num_heads))
        self.register_buffer("relative_position_index", _rel_index(window), persistent=True)
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        self._mask_cache = {}

    def _bias(self, pad_h, pad_w, shift, device, dtype):
        """[nW or 1, heads, N, N]: relative-position bias (+ -100 shift mask), cached per shape."""
        N = self.window * self.window
        rel = self.relative_position_bias_table[self.relative_position_index].view(N, N, -1)
        rel = rel.permute(2, 0, 1).contiguous().unsqueeze(0)                                   # [1, h, N, N]
        if shift == 0:
            return rel.to(dtype)
        key = (pad_h, pad_w, shift, device)
        m = self._mask_cache.get(key)
        if m is None:
            ws = self.window
            img = torch.zeros(pad_h, pad_w, device=device)
            cnt = 0
            for hs in ((0, -ws), (-ws, -shift), (-shift, None)):
                for wsl in ((0, -ws), (-ws, -shift), (-shift, None)):
                    img[hs[0]:hs[1], wsl[0]:wsl[1]] = cnt
                    cnt += 1
            win = img.view(pad_h // ws, ws, pad_w // ws, ws).permute(0, 2, 1, 3).reshape(-1, N)
            m = (win[:, :, None] - win[:, None, :]).ne(0).float() * -100.0                      # [nW, N, N]
            m = m.unsqueeze(1)
            self._mask_cache[key] = m
        return (rel + m).to(dtype)                                                             # [nW, h, N, N]

    def forward(self, x):  # x: [B, H, W, C]
        B, H, W, C = x.shape
        ws = self.window
        pr, pb = (ws - W % ws) % ws, (ws - H % ws) % ws
        x = F.pad(x, (0, 0, 0, pr, 0, pb))
        ph, pw = H + pb, W + pr
        shift = 0 if (ws >= ph and ws >= pw) else self.shift
        if shift > 0:
            x = torch.roll(x, shifts=(-shift, -shift), dims=(1, 2))
        nW = (ph // ws) * (pw // ws)
        x = x.view(B, ph // ws, ws, pw // ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B * nW, ws * ws, C)
        qkv = self.qkv(x).view(B * nW, ws * ws, 3, self.num_heads, C // self.num_heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]                                                       # [B nW, h, N, d]
        q = q * (C // self.num_heads) ** -0.5
        attn = q.matmul(k.transpose(-2, -1))
        bias = self._bias(ph, pw, shift, x.device, attn.dtype)
        attn = (attn.view(B, nW, self.num_heads, ws * ws, ws * ws) + bias.unsqueeze(0)).view_as(attn)
        attn = F.softmax(attn.float(), dim=-1).to(q.dtype)
        attn = F.dropout(attn, p=self.attention_dropout, training=self.training)
        x = attn.matmul(v).transpose(1, 2).reshape(B * nW, ws * ws, C)
        x = F.dropout(self.proj(x), p=self.dropout, training=self.training)
        x = x.view(B, ph // ws, pw // ws, ws, ws, C).permute(0, 1, 3, 2, 4, 5).reshape(B, ph, pw, C)
        if shift > 0:
            x = torch.roll(x, shifts=(shift, shift), dims=(1, 2))
        return x[:, :H, :W, :].contiguous()


class MLP(nn.Sequential):
    def __init__(self, dim, hidden, dropout=0.0):
        super().__init__(nn.Linear(dim, hidden), nn.GELU(), nn.Dropout(dropout), nn.Linear(hidden, dim),
                         nn.Dropout(dropout))


class SwinTransformerBlock(nn.Module):
    def __init__(self, dim, num_heads, window, shift, mlp_ratio=4.0, dropout=0.0, attention_dropout=0.0,
                 stochastic_depth_prob=0.0):
        super().__init__()
        self.norm1 = LayerNorm(dim, eps=1e-5)
        self.attn = ShiftedWindowAttention(dim, window, shift, num_heads, attention_dropout, dropout)
        self.sd = stochastic_depth_prob
        self.norm2 = LayerNorm(dim, eps=1e-5)
        self.mlp = MLP(dim, int(dim * mlp_ratio), dropout)

    def forward(self, x):
        x = x + _stochastic_depth(self.attn(self.norm1(x)), self.sd, self.training)
        return x + _stochastic_depth(self.mlp(self.norm2(x)), self.sd, self.training)


class PatchMerging(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.reduction = nn.Linear(4 * dim, 2 * dim, bias=False)
        self.norm = LayerNorm(4 * dim, eps=1e-5)

    def forward(self, x):  # [B, H, W, C] -> [B, H/2, W/2, 2C]
        H, W = x.shape[1], x.shape[2]
        x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2))
        x = torch.cat([x[:, 0::2, 0::2], x[:, 1::2, 0::2], x[:, 0::2, 1::2], x[:, 1::2, 1::2]], -1)
        return self.reduction(self.norm(x))


class Permute(nn.Module):
    def __init__(self, dims):
        super().__init__()
        self.dims = dims

    def forward(self, x):
        return x.permute(*self.dims)


class SwinTransformer(nn.Module):
    def __init__(self, embed_dim=96, depths=(2, 2, 6, 2), num_heads=(3, 6, 12, 24), window_size=7,
                 patch_size=4, mlp_ratio=4.0, dropout=0.0, attention_dropout=0.0, stochastic_depth_prob=0.1,
                 num_classes=1000):
        super().__init__()
        layers: List[nn.Module] = [nn.Sequential(
            nn.Conv2d(3, embed_dim, kernel_size=patch_size, stride=patch_size), Permute([0, 2, 3, 1]),
            LayerNorm(embed_dim, eps=1e-5))]
        total = sum(depths)
        bid = 0
        for i, depth in enumerate(depths):
            dim = embed_dim * 2 ** i
            stage = []
            for j in range(depth):
                sd = stochastic_depth_prob * bid / max(total - 1, 1)
                stage.append(SwinTransformerBlock(dim, num_heads[i], window_size, 0 if j % 2 == 0 else window_size // 2,
                                                  mlp_ratio, dropout, attention_dropout, sd))
                bid += 1
            layers.append(nn.Sequential(*stage))
            if i < len(depths) - 1:
                layers.append(PatchMerging(dim))
        self.features = nn.Sequential(*layers)
        nf = embed_dim * 2 ** (len(depths) - 1)
        self.norm = LayerNorm(nf, eps=1e-5)
        self.permute = Permute([0, 3, 1, 2])
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.flatten = nn.Flatten(1)
        self.head = nn.Linear(nf, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.trunc_normal_(m.weight, std=0.02)
                if m.bias is not None:
                    nn.init.zeros_(m.bias)

    def forward(self, x):  # NCHW (or channels_last) images
        x = self.features(x)
        x = self.norm(x)
        x = self.permute(x)
        x = self.avgpool(x)
        return self.head(self.flatten(x))


def swin(name: str, num_classes: int = 1000, **over) -> SwinTransformer:
    cfg = dict(CONFIGS[name])
    cfg.update(over)
    return SwinTransformer(num_classes=num_classes, **cfg)


def available():
    return sorted(CONFIGS)
