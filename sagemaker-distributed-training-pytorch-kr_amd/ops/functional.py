"""Autograd-aware fused ops backed by the gfx950 kernel library.

Every op has two paths:
  * GPU tensors -> the HIP kernels in ``smdt_amd/_C.so`` (no silent fallback: see ``_ext``);
  * CPU tensors -> a plain PyTorch reference with identical semantics (tests, gloo runs).

Reference-parity notes: these cover Megatron's fused kernels K1-K6, K12, K15,
K16 (`megatron/arguments.py:814-854` in /root/reference/3_training_megatron-lm) with the same
enable/disable flags wired up in ``smdt_amd.models.transformer``.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _ext

# --------------------------------------------------------------------------------------------
# Dropout RNG: stateless Philox (seed, offset) pairs. The forward call records its pair in the
# autograd context and the backward kernel regenerates the identical mask.


class PhiloxState:
    """Per-process (seed, offset) source for the fused dropout kernels.

    ``offset`` advances by one per kernel call, so successive calls draw independent streams.
    Tensor-parallel-aware seeding lives in ``smdt_amd.parallel.random``.
    """

    def __init__(self, seed: int = 1234):
        self.seed = int(seed)
        self.offset = 0

    def next(self):
        self.offset += 1
        return self.seed, self.offset

    def state_dict(self):
        return {"seed": self.seed, "offset": self.offset}

    def load_state_dict(self, d):
        self.seed, self.offset = int(d["seed"]), int(d["offset"])


_DEFAULT_RNG = PhiloxState()


def default_rng() -> PhiloxState:
    return _DEFAULT_RNG


def _rng(rng: Optional[PhiloxState]) -> PhiloxState:
    return rng if rng is not None else _DEFAULT_RNG


# --------------------------------------------------------------------------------------------
# Fused (bias + dropout + residual) -> LayerNorm / RMSNorm


def _ln_ref(s, gamma, beta, eps, rms):
    sf = s.float()
    if rms:
        y = sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()
    else:
        y = F.layer_norm(sf, (s.shape[-1],), gamma.float(), None if beta is None else beta.float(), eps)
    return y.to(s.dtype)


def grad_accumulate_target(t):
    """The fp32 DDP ``main_grad`` of parameter ``t`` if a kernel may accumulate the parameter's
    gradient straight into it (then the kernel owner calls ``t._smdt_grad_ready``), else None."""
    if t is None or not isinstance(t, torch.nn.Parameter):
        return None
    mg = getattr(t, "main_grad", None)
    if (mg is None or mg.dtype != torch.float32 or not mg.is_cuda or not mg.is_contiguous()
            or getattr(t, "_smdt_grad_ready", None) is None):
        return None
    return mg


def _mark_ready(*params):
    for t in params:
        if t is not None:
            t._smdt_grad_ready(t)


def gather_slot(t, world: int, rank: int):
    """A [world * n, ...] buffer (uninitialised) and its rank-th row block, the slot ``t``'s
    producer writes into so that a sequence-parallel all-gather of it needs no local copy
    (``tensor_parallel.ag_ring`` takes the buffer, marked on the slot as ``_smdt_gather``)."""
    n = t.shape[0]
    buf = t.new_empty((world * n,) + tuple(t.shape[1:]))
    return buf, buf[rank * n:(rank + 1) * n]


def _mark_gather(t, buf, rank):
    t._smdt_gather = (buf, rank)
    return t


class _BDALayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, residual, gamma, beta, p, eps, rms, seed, offset, gather=None, x2=None):
        """``gather`` = (world, rank, y_into_gather, dx_into_gather) under sequence parallelism:
        the normalised output (consumed by a column-parallel ring all-gather) and / or the input
        gradient (consumed by a row-parallel linear's backward all-gather) are written into their
        rank's slot of a gather buffer. ``x2`` (no gradient): a second summand of x, added in the
        kernel (a reduce-scatter's incoming partial, see ``tensor_parallel.rs_ring``); x's
        gradient is also x + x2's."""
        C = _ext.ext()
        x = x.contiguous()
        buf = out_y = None
        if gather is not None and gather[2]:
            buf, out_y = gather_slot(x, gather[0], gather[1])
        y, s, mean, rstd = C.layernorm_fwd(x, None if residual is None else residual.contiguous(),
                                           bias, gamma, beta, eps, p, seed, offset, rms, True, out_y,
                                           None if x2 is None else x2.contiguous())
        if buf is not None:
            _mark_gather(y, buf, gather[1])
        ctx.save_for_backward(s, gamma, mean, rstd)
        ctx.pref = (bias, gamma, beta)  # parameter objects: their main_grad / readiness hooks
        ctx.cfg = (p, seed, offset, rms, bias is not None, residual is not None, beta is not None,
                   gamma.dtype, None if bias is None else bias.dtype)
        ctx.gather = gather
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, gamma, mean, rstd = ctx.saved_tensors
        p, seed, offset, rms, has_bias, has_res, has_beta, gdt, bdt = ctx.cfg
        C = _ext.ext()
        # the consuming column-parallel linear's backward reduce-scatter may leave its peer's
        # partial as a pending summand of dy (tensor_parallel.rs_ring, defer_add): added in-kernel
        from ..parallel.tensor_parallel import take_pending_add
        dy2 = take_pending_add(dy)
        dy = dy.contiguous()
        ds = None if ds is None else ds.contiguous()
        bias_p, gamma_p, beta_p = ctx.pref
        # bias / gamma / beta gradients go straight into fp32 main_grad when DDP owns them
        ta = grad_accumulate_target(gamma_p)
        tb = grad_accumulate_target(beta_p) if has_beta else None
        tc = grad_accumulate_target(bias_p) if has_bias else None
        gbuf = out_dx = None
        if ctx.gather is not None and ctx.gather[3]:
            gbuf, out_dx = gather_slot(s, ctx.gather[0], ctx.gather[1])
        d_s, dx, dgamma, dbeta, dbias = C.layernorm_bwd(dy, ds, s, gamma, mean, rstd, p, seed, offset, rms,
                                                        True, has_bias, ta, tb, tc, out_dx,
                                                        None if dy2 is None else dy2.contiguous())
        if gbuf is not None:
            _mark_gather(dx, gbuf, ctx.gather[1])
        _mark_ready(gamma_p if ta is not None else None, beta_p if tb is not None else None,
                    bias_p if tc is not None else None)
        g_gamma = None if ta is not None else dgamma.to(gdt)
        g_beta = None if (not has_beta or tb is not None) else dbeta.to(gdt)
        g_bias = None if (not has_bias or tc is not None) else dbias.to(bdt)
        return (dx, g_bias, d_s if has_res else None, g_gamma, g_beta, None, None, None, None, None, None, None)


def bias_dropout_add_norm(x, bias, residual, gamma, beta, p: float, training: bool, eps: float = 1e-5,
                          rms: bool = False, rng: Optional[PhiloxState] = None, gather=None):
    """Returns ``(norm(s), s)`` with ``s = residual + dropout(x + bias)``.

    ``bias``, ``residual`` may be None; ``beta`` is ignored for RMSNorm. This is the
    residual-stream step of a pre-LN transformer fused with the following LayerNorm.
    ``gather`` (world, rank, y, dx): see ``_BDALayerNorm.forward`` (kernel path only).
    """
    p = float(p) if training else 0.0
    # a row-parallel output whose reduce-scatter left its peer's partial as a pending summand
    # (tensor_parallel.rs_ring under defer_rs_add): x + x2 is the value, added in the kernel
    from ..parallel.tensor_parallel import plain, take_pending_add
    x2 = take_pending_add(x)
    x = plain(x)
    if _ext.use_kernels(x):
        seed, offset = _rng(rng).next() if p > 0 else (0, 0)
        return _BDALayerNorm.apply(x, bias, residual, gamma, None if rms else beta, p, float(eps), bool(rms),
                                   int(seed), int(offset), gather, x2)
    if x2 is not None:
        x = x + x2
    h = x if bias is None else x + bias
    if p > 0:
        h = F.dropout(h, p=p, training=True)
    s = h if residual is None else residual + h
    if rms:
        sf = s.float()
        y = (sf * torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps) * gamma.float()).to(s.dtype)
    else:
        y = F.layer_norm(s.float(), (s.shape[-1],), gamma.float(), None if beta is None else beta.float(),
                         eps).to(s.dtype)
    return y, s


def layer_norm(x, gamma, beta, eps: float = 1e-5):
    return bias_dropout_add_norm(x, None, None, gamma, beta, 0.0, False, eps, False)[0]


def rms_norm(x, gamma, eps: float = 1e-6):
    return bias_dropout_add_norm(x, None, None, gamma, None, 0.0, False, eps, True)[0]


def bias_dropout_add(x, bias, residual, p: float, training: bool):
    """Unfused residual step (pipeline-stage boundaries only)."""
    h = x if bias is None else x + bias
    if training and p > 0:
        h = F.dropout(h, p=p, training=True)
    return h if residual is None else residual + h


# --------------------------------------------------------------------------------------------
# bias + GeLU / SwiGLU

_ACT_CODES = {"gelu": 0, "gelu_tanh": 0, "gelu_erf": 1}


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act):
        C = _ext.ext()
        x = x.contiguous()
        y = C.bias_act_fwd(x, bias, act)
        ctx.save_for_backward(x, bias)
        ctx.bias_p = bias
        ctx.act = act
        ctx.has_bias = bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        C = _ext.ext()
        # a detached bias (ColumnParallelLinear(bias_grad_from_output=True): the linear produces
        # the bias gradient with its weight gradient) needs no column sums here
        want_db = ctx.has_bias and ctx.needs_input_grad[1]
        tgt = grad_accumulate_target(ctx.bias_p) if want_db else None
        dx, dbias = C.bias_act_bwd(dy.contiguous(), x, bias, ctx.act, want_db, tgt)
        if tgt is not None:
            _mark_ready(ctx.bias_p)
            return dx, None, None
        return dx, (dbias.to(bias.dtype) if want_db else None), None


def bias_gelu(x, bias=None, approximate: str = "tanh"):
    """GeLU(x + bias); ``approximate='tanh'`` is Megatron's bias_gelu, 'none' the erf form."""
    act = 0 if approximate == "tanh" else 1
    if _ext.use_kernels(x):
        return _BiasAct.apply(x, bias, act)
    h = x if bias is None else x + bias
    return F.gelu(h.float(), approximate="tanh" if act == 0 else "none").to(x.dtype)


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        C = _ext.ext()
        x = x.contiguous()
        ctx.save_for_backward(x)
        return C.swiglu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return _ext.ext().swiglu_bwd(dy.contiguous(), x)


def swiglu(x):
    """x = [gate | up] on the last dim -> silu(gate) * up."""
    if _ext.use_kernels(x):
        return _SwiGLU.apply(x)
    g, u = x.chunk(2, dim=-1)
    return (F.silu(g.float()) * u.float()).to(x.dtype)


# --------------------------------------------------------------------------------------------
# Scaled masked softmax (Megatron K1-K3)


class _ScaledSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask, mode, scale):
        C = _ext.ext()
        y = C.softmax_fwd(x.contiguous(), mask, mode, scale)
        ctx.save_for_backward(y)
        ctx.mode, ctx.scale = mode, scale
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return _ext.ext().softmax_bwd(dy.contiguous(), y, ctx.mode, ctx.scale), None, None, None


def scaled_masked_softmax(x, mask=None, scale: float = 1.0, causal: bool = False):
    """softmax(scale * x) over the last dim of [b, np, sq, sk].

    ``causal`` masks key j > query i (Megatron's upper-triangular mask); otherwise ``mask``
    ([b, 1, sq, sk] bool, True = masked) is applied if given.
    """
    mode = 1 if causal else (2 if mask is not None else 0)
    if _ext.use_kernels(x) and x.shape[-1] <= 4096 and x.shape[-1] % 8 == 0:
        m = None
        if mode == 2:
            m = mask.expand(x.shape[0], 1, x.shape[2], x.shape[3]).contiguous().to(torch.uint8)
        return _ScaledSoftmax.apply(x, m, mode, float(scale))
    xf = x.float() * scale
    if mode == 1:
        sq, sk = x.shape[-2], x.shape[-1]
        cm = torch.ones(sq, sk, dtype=torch.bool, device=x.device).triu(1 + sk - sq)
        xf = xf.masked_fill(cm, float("-inf"))
    elif mode == 2:
        xf = xf.masked_fill(mask, float("-inf"))
    y = torch.softmax(xf, dim=-1)
    y = torch.nan_to_num(y, nan=0.0)
    return y.to(x.dtype)


# --------------------------------------------------------------------------------------------
# Flash attention


def _qkv_views(qkv, nh, nkv, hd, seq_first):
    """[S, B, W] (seq_first) or [B, S, W] fused projection output -> q, k, v as [B, S, H, D]
    views with W = (nh + 2 nkv) hd laid out as [q heads | k heads | v heads]."""
    if seq_first:
        x = qkv.transpose(0, 1)
    else:
        x = qkv
    q = x[..., : nh * hd].unflatten(-1, (nh, hd))
    k = x[..., nh * hd:(nh + nkv) * hd].unflatten(-1, (nkv, hd))
    v = x[..., (nh + nkv) * hd:].unflatten(-1, (nkv, hd))
    return q, k, v


class _FlashAttnQKV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, nh, nkv, hd, seq_first, scale, causal, dropout_p=0.0, seed=0, offset=0):
        C = _ext.ext()
        q, k, v = _qkv_views(qkv, nh, nkv, hd, seq_first)
        if seq_first:
            S, B = qkv.shape[0], qkv.shape[1]
            out = qkv.new_empty(S, B, nh, hd)
            ov = out.transpose(0, 1)
        else:
            B, S = qkv.shape[0], qkv.shape[1]
            out = qkv.new_empty(B, S, nh, hd)
            ov = out
        _, lse = C.flash_fwd(q, k, v, scale, causal, ov, dropout_p, seed, offset)
        ctx.save_for_backward(qkv, out, lse)
        ctx.cfg = (nh, nkv, hd, seq_first, scale, causal, dropout_p, seed, offset)
        return out.flatten(-2)

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        nh, nkv, hd, seq_first, scale, causal, dropout_p, seed, offset = ctx.cfg
        C = _ext.ext()
        q, k, v = _qkv_views(qkv, nh, nkv, hd, seq_first)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _qkv_views(dqkv, nh, nkv, hd, seq_first)
        do = dout.unflatten(-1, (nh, hd))
        o = out
        if seq_first:
            do = do.transpose(0, 1)
            o = o.transpose(0, 1)
        C.flash_bwd(q, k, v, o, do, lse, scale, causal, dq, dk, dv, dropout_p, seed, offset)
        return dqkv, None, None, None, None, None, None, None, None, None


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, scale, causal, dropout_p=0.0, seed=0, offset=0):
        C = _ext.ext()
        o, lse = C.flash_fwd(q, k, v, scale, causal, None, dropout_p, seed, offset)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (scale, causal, dropout_p, seed, offset)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        scale, causal, p, seed, offset = ctx.cfg
        dq, dk, dv = _ext.ext().flash_bwd(q, k, v, o, do, lse, scale, causal, None, None, None, p, seed, offset)
        return dq, dk, dv, None, None, None, None, None


_M32 = 0xFFFFFFFF


def _fmix32_t(x):
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & _M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & _M32
    return x ^ (x >> 16)


def _fmix32_i(x: int) -> int:
    x &= _M32
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & _M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & _M32
    return x ^ (x >> 16)


def flash_dropout_thr(p: float):
    """(7-bit threshold, keep scale) the kernels use for drop probability ``p``: the realised drop
    rate is round(p * 128) / 128 (the kernels test the low 7 bits of each random byte with one
    SWAR add per 4 bytes; FlashAttention-2 thresholds random bytes too)."""
    thr = min(int(p * 128.0 + 0.5), 127)
    return thr, 128.0 / (128.0 - thr)


# Graph-safe dropout RNG. The fused dropout kernels take a (seed, offset) pair per call from the
# host (``_Rng``); inside a captured HIP graph those values are baked into the kernel arguments
# and every replay would redraw the same masks. With a device step counter registered, every
# dropout kernel mixes the counter's value into its key at run time (flash_attn.hip drop_key,
# layernorm.hip ln_drop_key); ``advance_graph_rng`` (a device add, captured with the step)
# moves it once per training step — after the backward, so forward and backward of a step see
# the same masks.
_GRAPH_RNG = {"counter": None}


def enable_graph_rng(device=None) -> torch.Tensor:
    c = _GRAPH_RNG["counter"]
    if c is None:
        c = torch.zeros(1, dtype=torch.int32, device=device or torch.device("cuda", torch.cuda.current_device()))
        _ext.ext().set_rng_step(c)
        _GRAPH_RNG["counter"] = c
    return c


def disable_graph_rng():
    if _GRAPH_RNG["counter"] is not None:
        _ext.ext().set_rng_step(None)
        _GRAPH_RNG["counter"] = None


def advance_graph_rng():
    c = _GRAPH_RNG["counter"]
    if c is not None:
        c.add_(1)


def flash_dropout_keep_mask(B: int, H: int, S: int, p: float, seed: int, offset: int, device=None,
                            step: Optional[int] = None):
    """Bit-exact twin of the flash kernels' dropout mask: bool [B, H, S(q), S(k)], True = kept
    (see ``drop_hash`` in flash_attn.hip): each 2x2 (query, key) block shares one hash, byte
    2 (q & 1) + (k & 1) decides the element (kept iff its low 7 bits >= the threshold).
    ``step``: the graph-safe RNG counter value the kernels read (``enable_graph_rng``)."""
    thr, _ = flash_dropout_thr(p)
    key0 = _fmix32_i((seed & _M32) ^ _fmix32_i(((seed >> 32) + 0x9E3779B9) & _M32))
    key1 = _fmix32_i((((offset & _M32) * 0x27D4EB2F) & _M32) ^ _fmix32_i(((offset >> 32) + 0x165667B1) & _M32))
    if step is not None:
        key1 ^= _fmix32_i(((step & _M32) * 0x9E3779B1 + 0x85EBCA77) & _M32)
    bh = torch.arange(B * H, dtype=torch.int64, device=device)
    kbh = _fmix32_t((key0 + bh * 0x632BE5AB) & _M32) ^ key1                          # [BH]
    half = S // 2
    blk = (torch.arange(half, dtype=torch.int64, device=device)[:, None] * half
           + torch.arange(half, dtype=torch.int64, device=device)[None, :])            # [S/2, S/2]
    x = blk[None] ^ kbh[:, None, None]
    x = (((x ^ (x >> 16)) & 0xFFFFFF) * 0x45D9F3) & _M32   # v_mul_u32_u24
    x = (((x ^ (x >> 16)) & 0xFFFFFF) * 0x45D9F3) & _M32
    x = x ^ (x >> 16)
    by = torch.stack([(x >> (8 * i)) & 0x7F for i in range(4)], dim=-1) >= thr           # [BH, S/2, S/2, 4]
    # byte 2 qb + kb -> [BH, S/2, S/2, 2(q), 2(k)] -> [BH, S/2, 2, S/2, 2]
    keep = by.view(B * H, half, half, 2, 2).permute(0, 1, 3, 2, 4)
    return keep.reshape(B, H, S, S)


def attention_ref(q, k, v, scale, causal, dropout_p: float = 0.0, keep=None):
    """Reference attention on [B, S, H, D] (GQA by head repetition), fp32 math. ``keep``
    ([B, H, S, S] bool) is the dropout keep-mask (``flash_dropout_keep_mask``)."""
    if q.is_cuda and os.environ.get("SMDT_ASSERT_FLASH") == "1":
        raise RuntimeError("SMDT_ASSERT_FLASH=1: reference attention reached on the GPU")
    B, S, H, D = q.shape
    Hkv = k.shape[2]
    if Hkv != H:
        k = k.repeat_interleave(H // Hkv, dim=2)
        v = v.repeat_interleave(H // Hkv, dim=2)
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        cm = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(cm, float("-inf"))
    p = torch.softmax(s, dim=-1)
    if dropout_p > 0:
        if keep is None:
            p = torch.nn.functional.dropout(p, dropout_p, training=True)
        else:
            p = p * keep * flash_dropout_thr(dropout_p)[1]
    o = torch.matmul(p, vf).transpose(1, 2)
    return o.to(q.dtype)


def flash_supported(q, k) -> bool:
    """True when the kernels take q / k exactly as they are (no padding)."""
    B, S, H, D = q.shape
    return (q.dtype in (torch.bfloat16, torch.float16) and D in (64, 128) and S % 128 == 0
            and H % k.shape[2] == 0 and q.stride(-1) == 1 and k.stride(-1) == 1)


def _flash_plan(q, k, causal: bool):
    """(S_pad, D_pad) the gfx950 kernels run this attention at, or raise — a GPU tensor never
    drops to the materialised S x S reference (ops/_ext.py policy).

    Padding is exact where it is used: head dims below 64 / 128 are zero-padded (zero q / k
    columns add nothing to q.k, zero v columns produce output columns that are sliced off, and
    the softmax scale stays 1 / sqrt(D_orig)); a causal sequence is padded at its END (no real
    query attends to a later key). A non-causal sequence that is not a multiple of 128 would
    need key masking and is rejected."""
    B, S, H, D = q.shape
    if q.dtype not in (torch.bfloat16, torch.float16):
        raise RuntimeError(f"flash attention on the GPU runs bf16 / fp16, got {q.dtype}; cast the model "
                           "(--bf16 / --fp16) or disable flash attention (--no-flash-attn)")
    if H % k.shape[2]:
        raise RuntimeError(f"flash attention: {H} query heads are not a multiple of {k.shape[2]} kv heads")
    if D > 128:
        raise RuntimeError(f"flash attention: head dim {D} > 128 is not supported by the gfx950 kernels")
    Dp = 64 if D <= 64 else 128
    Sp = -(-S // 128) * 128
    if Sp != S and not causal:
        raise RuntimeError(f"flash attention: non-causal sequence length {S} must be a multiple of 128")
    return Sp, Dp


def _pad_bshd(t, Sp, Dp):
    S, D = t.shape[1], t.shape[3]
    if Sp == S and Dp == D:
        return t
    return torch.nn.functional.pad(t, (0, Dp - D, 0, 0, 0, Sp - S))


def flash_attention(q, k, v, scale: Optional[float] = None, causal: bool = True, dropout_p: float = 0.0,
                    rng: Optional[PhiloxState] = None):
    """Attention over [B, S, H, D] tensors (any batch/seq/head strides, unit last stride);
    ``k``/``v`` may have fewer heads (GQA)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    seed, off = _rng(rng).next() if dropout_p > 0 else (0, 0)
    if _ext.use_kernels(q):
        S, D = q.shape[1], q.shape[3]
        Sp, Dp = _flash_plan(q, k, causal)
        if (Sp, Dp) == (S, D) and flash_supported(q, k):
            return _FlashAttn.apply(q, k, v, float(scale), bool(causal), float(dropout_p), int(seed), int(off))
        qp, kp, vp = (_pad_bshd(t.contiguous() if t.stride(-1) != 1 else t, Sp, Dp) for t in (q, k, v))
        o = _FlashAttn.apply(qp, kp, vp, float(scale), bool(causal), float(dropout_p), int(seed), int(off))
        return o[:, :S, :, :D]
    keep = flash_dropout_keep_mask(q.shape[0], q.shape[2], q.shape[1], dropout_p, seed, off, q.device) \
        if dropout_p > 0 else None
    return attention_ref(q, k, v, scale, causal, dropout_p, keep)


def flash_attention_qkv(qkv, nh: int, nkv: int, hd: int, seq_first: bool = True, causal: bool = True,
                        scale: Optional[float] = None, dropout_p: float = 0.0, rng: Optional[PhiloxState] = None):
    """Attention straight off a fused QKV projection output.

    ``qkv`` is [S, B, (nh + 2 nkv) hd] (``seq_first``) or [B, S, ...]; returns [S, B, nh hd]
    (resp. [B, S, nh hd]). Backward produces ONE fused d(qkv) buffer. ``dropout_p`` > 0 applies
    attention-probability dropout inside the kernels (mask re-derived from ``rng``'s
    (seed, offset) in backward — nothing is stored). Shapes the kernels cannot read in place
    (S % 128 != 0, head dim not 64 / 128) go through the padded separate-q/k/v path.
    """
    if scale is None:
        scale = 1.0 / math.sqrt(hd)
    q, k, v = _qkv_views(qkv, nh, nkv, hd, seq_first)
    if _ext.use_kernels(qkv):
        if qkv.is_contiguous() and flash_supported(q, k) and (nh + 2 * nkv) * hd % 8 == 0:
            seed, off = _rng(rng).next() if dropout_p > 0 else (0, 0)
            return _FlashAttnQKV.apply(qkv, nh, nkv, hd, bool(seq_first), float(scale), bool(causal),
                                       float(dropout_p), int(seed), int(off))
        o = flash_attention(q, k, v, scale, causal, dropout_p, rng)          # [B, S, H, D]
    else:
        seed, off = _rng(rng).next() if dropout_p > 0 else (0, 0)
        keep = None
        if dropout_p > 0:
            keep = flash_dropout_keep_mask(q.shape[0], nh, q.shape[1], dropout_p, seed, off, qkv.device)
        o = attention_ref(q, k, v, scale, causal, dropout_p, keep)  # [B, S, H, D]
    if seq_first:
        o = o.transpose(0, 1)
    return o.flatten(-2).contiguous()


# --------------------------------------------------------------------------------------------
# Rotary embedding


def rope_tables(max_pos: int, rot_dim: int, base: float = 10000.0, device=None):
    inv = 1.0 / (base ** (torch.arange(0, rot_dim, 2, dtype=torch.float64) / rot_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device), f.sin().float().to(device)


def _rope_ref(x, cos, sin, rot, pos, inverse=False):
    # x [ntok, nh, d]; pos [ntok]
    xr = x[..., :rot].float()
    x1, x2 = xr[..., : rot // 2], xr[..., rot // 2:]
    c = cos[pos].unsqueeze(1)
    s = sin[pos].unsqueeze(1)
    if inverse:
        s = -s
    out = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)
    return torch.cat([out, x[..., rot:]], dim=-1) if rot < x.shape[-1] else out


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, rot, pos_div, pos_mod):
        y = x.clone()
        _ext.ext().rope_(y, cos, sin, rot, pos_div, pos_mod, False)
        ctx.save_for_backward(cos, sin)
        ctx.cfg = (rot, pos_div, pos_mod)
        return y

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        rot, pos_div, pos_mod = ctx.cfg
        dx = dy.contiguous().clone()
        _ext.ext().rope_(dx, cos, sin, rot, pos_div, pos_mod, True)
        return dx, None, None, None, None, None


def apply_rope(x, cos, sin, pos_div: int, pos_mod: int, rot: Optional[int] = None):
    """Rotate-half RoPE on x [ntok, nh, d]; token t has position (t // pos_div) % pos_mod."""
    rot = rot or x.shape[-1]
    if _ext.use_kernels(x) and rot % 16 == 0:
        xx = x if x.stride(-1) == 1 and x.stride(0) % 8 == 0 and x.stride(1) % 8 == 0 else x.contiguous()
        return _Rope.apply(xx, cos, sin, rot, pos_div, pos_mod)
    pos = (torch.arange(x.shape[0], device=x.device) // pos_div) % pos_mod
    return _rope_ref(x, cos.to(x.device), sin.to(x.device), rot, pos)


# --------------------------------------------------------------------------------------------
# (Vocab-parallel) cross entropy


class _FusedCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, vstart, group, ignore_index, inplace_grad, vvalid):
        C = _ext.ext()
        lg = logits.contiguous()
        t = target.contiguous().view(-1)
        mx, se, tg = C.ce_stats(lg.view(-1, lg.shape[-1]), t, vstart, vvalid)
        if group is not None and torch.distributed.get_world_size(group) > 1:
            from ..comm import stats as _cs
            gmax = mx.clone()
            with _cs.blocking("all_reduce", group, 3 * gmax.numel() * gmax.element_size()):
                torch.distributed.all_reduce(gmax, op=torch.distributed.ReduceOp.MAX, group=group)
                se = se * torch.exp(mx - gmax)
                torch.distributed.all_reduce(se, group=group)
                torch.distributed.all_reduce(tg, group=group)
            mx = gmax
        loss = torch.log(se) + mx - tg
        loss = torch.where(t == ignore_index, torch.zeros_like(loss), loss)
        ctx.save_for_backward(lg, t, mx, se)
        ctx.cfg = (vstart, ignore_index, inplace_grad, vvalid)
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, dloss):
        lg, t, mx, se = ctx.saved_tensors
        vstart, ignore_index, inplace_grad, vvalid = ctx.cfg
        C = _ext.ext()
        out = lg if inplace_grad else torch.empty_like(lg)
        C.ce_bwd(lg.view(-1, lg.shape[-1]), t, mx, se, dloss.contiguous().view(-1).float(),
                 out.view(-1, lg.shape[-1]), vstart, ignore_index, vvalid)
        return out, None, None, None, None, None, None


def cross_entropy(logits, target, vocab_start: int = 0, group=None, ignore_index: int = -100,
                  inplace_grad: bool = False, vocab_size: int = 0):
    """Per-token CE loss (fp32) for logits [..., V_local] holding vocab slice
    [vocab_start, vocab_start + V_local). With ``group`` the logits are vocab-parallel and the
    three per-row statistics are all-reduced (MAX, SUM, SUM) across it.

    ``inplace_grad=True`` writes dlogits over the logits buffer (saves a [tokens, V] tensor);
    only valid when nothing else reads the logits after the loss.
    ``vocab_size`` > 0 marks global columns >= vocab_size as padding (excluded from the softmax,
    zero gradient) — HF semantics for a vocab padded to a multiple of 128.
    """
    vvalid = 0
    if vocab_size > 0:
        vvalid = min(max(int(vocab_size) - int(vocab_start), 0), logits.shape[-1])
        assert vvalid > 0, "a vocab shard holds only padding; use a smaller padding multiple"
        if vvalid == logits.shape[-1]:
            vvalid = 0
    if _ext.use_kernels(logits) and logits.shape[-1] % 8 == 0:
        return _FusedCE.apply(logits, target, int(vocab_start), group, int(ignore_index), bool(inplace_grad),
                              vvalid)
    return _ce_ref(logits, target, vocab_start, group, ignore_index, vvalid)


class _CERef(torch.autograd.Function):
    """Vocab-parallel CE in plain PyTorch (CPU path), same math as the fused kernel."""

    @staticmethod
    def forward(ctx, logits, target, vstart, group, ignore_index, vvalid=0):
        lf = logits.float()
        V = lf.shape[-1]
        if vvalid:
            lf = lf.clone()
            lf[..., vvalid:] = float("-inf")
        mx = lf.max(-1).values
        ws = 1
        if group is not None:
            ws = torch.distributed.get_world_size(group)
        if ws > 1:
            torch.distributed.all_reduce(mx, op=torch.distributed.ReduceOp.MAX, group=group)
        ex = torch.exp(lf - mx.unsqueeze(-1))
        se = ex.sum(-1)
        local = target - vstart
        inr = (local >= 0) & (local < V)
        idx = local.clamp(0, V - 1)
        tg = torch.gather(lf, -1, idx.unsqueeze(-1)).squeeze(-1) * inr
        if ws > 1:
            torch.distributed.all_reduce(se, group=group)
            torch.distributed.all_reduce(tg, group=group)
        loss = torch.log(se) + mx - tg
        ign = target == ignore_index
        loss = loss.masked_fill(ign, 0.0)
        ctx.save_for_backward(ex, se, idx, inr, ign)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        ex, se, idx, inr, ign = ctx.saved_tensors
        p = ex / se.unsqueeze(-1)
        oh = torch.zeros_like(p).scatter_(-1, idx.unsqueeze(-1), inr.unsqueeze(-1).float())
        d = (p - oh) * g.masked_fill(ign, 0.0).unsqueeze(-1)
        return d.to(ctx.dtype), None, None, None, None, None


def _ce_ref(logits, target, vocab_start, group, ignore_index, vvalid=0):
    return _CERef.apply(logits, target, int(vocab_start), group, int(ignore_index), int(vvalid))
