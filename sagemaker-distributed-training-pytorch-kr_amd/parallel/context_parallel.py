"""Context parallelism for long sequences: Ulysses-style all-to-all attention over a CP group.

SURVEY P10 / §5.7: the reference has no context parallelism (no ``--context-parallel-size`` in
/root/reference/3_training_megatron-lm/megatron/arguments.py; its longest context is the
``--seq-length`` / ``--max-position-embeddings`` limit at :569-571, :1124-1125). This module is the
optional long-context stretch.

Why all-to-all (Ulysses) rather than a K/V ring on MI355X: the 8 GPUs of a node form a fully
connected xGMI mesh (7 point-to-point links per GPU). A ring pass uses ONE link per step and needs
cp-1 dependent steps; an all-to-all drives all cp-1 links at once, moving each activation byte
once. Each rank holds ``s/cp`` tokens of every head outside attention; the all-to-all re-shards to
the FULL sequence for ``nh/cp`` heads, so the unchanged flash-attention kernel (causal skip,
dropout, GQA) runs on a full-length problem, and a second all-to-all shards the output back.
Backward is the mirror image (each all-to-all's adjoint is the opposite all-to-all).

Layout: activations are sequence-first [s_local, b, heads, d] (the transformer's [s, b, h]
layout), rank r holding the contiguous sequence chunk r.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..ops import functional as SF


def _a2a(x: torch.Tensor, group) -> torch.Tensor:
    """all_to_all_single along dim 0 (chunk j goes to rank j, chunk i of the result came from i)."""
    x = x.contiguous()
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x, group=group)
    return out


def _seq_to_head(x: torch.Tensor, group) -> torch.Tensor:
    """[s/cp, b, nh, d] (sequence-sharded) -> [s, b, nh/cp, d] (head-sharded)."""
    cp = dist.get_world_size(group)
    sl, b, nh, d = x.shape
    assert nh % cp == 0, f"{nh} heads not divisible by context-parallel size {cp}"
    # chunk j = head group j of my sequence chunk -> rank j
    send = x.reshape(sl, b, cp, nh // cp, d).permute(2, 0, 1, 3, 4)
    recv = _a2a(send, group)                      # chunk i = sequence chunk i of my head group
    return recv.view(cp * sl, b, nh // cp, d)


def _head_to_seq(x: torch.Tensor, group) -> torch.Tensor:
    """[s, b, nh/cp, d] (head-sharded) -> [s/cp, b, nh, d] (sequence-sharded)."""
    cp = dist.get_world_size(group)
    s, b, nhl, d = x.shape
    assert s % cp == 0, f"sequence {s} not divisible by context-parallel size {cp}"
    recv = _a2a(x.reshape(cp, s // cp, b, nhl, d), group)   # chunk i = head group i of my sequence chunk
    return recv.permute(1, 2, 0, 3, 4).reshape(s // cp, b, cp * nhl, d)


class _SeqToHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _seq_to_head(x, group)

    @staticmethod
    def backward(ctx, g):
        return _head_to_seq(g, ctx.group), None


class _HeadToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _head_to_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _seq_to_head(g, ctx.group), None


def seq_to_head(x, group):
    return _SeqToHead.apply(x, group)


def head_to_seq(x, group):
    return _HeadToSeq.apply(x, group)


def ulysses_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group=None, causal: bool = True,
                      scale: Optional[float] = None, dropout_p: float = 0.0, rng=None,
                      attn_fn: Optional[Callable] = None) -> torch.Tensor:
    """Attention over a sequence sharded across ``group``.

    ``q`` is [s/cp, b, nh, d]; ``k``/``v`` are [s/cp, b, nkv, d]. GQA: if ``nkv`` is not a
    multiple of cp the K/V heads are replicated (to ``cp`` heads if that keeps the q->kv grouping,
    else to ``nh``) before the exchange. Returns [s/cp, b, nh, d]. ``attn_fn(q, k, v)`` takes and
    returns [b, s, heads, d] tensors; default is the gfx950 flash attention (PyTorch reference on
    CPU). Each rank attends over different heads, so pass a per-CP-rank ``rng`` for dropout.
    """
    group = group if group is not None else dist.group.WORLD
    cp = dist.get_world_size(group)
    nh, nkv = q.shape[2], k.shape[2]
    if nkv % cp != 0:
        rep = cp // nkv if (cp % nkv == 0 and (nh // nkv) % (cp // nkv) == 0) else nh // nkv
        k = k.repeat_interleave(rep, dim=2)
        v = v.repeat_interleave(rep, dim=2)
    if cp == 1:
        qh, kh, vh = q, k, v
    else:
        qh, kh, vh = seq_to_head(q, group), seq_to_head(k, group), seq_to_head(v, group)
    if attn_fn is None:
        def attn_fn(a, b_, c):
            return SF.flash_attention(a, b_, c, scale=scale, causal=causal, dropout_p=dropout_p, rng=rng)
    out = attn_fn(qh.transpose(0, 1), kh.transpose(0, 1), vh.transpose(0, 1)).transpose(0, 1)  # [s, b, nh/cp, d]
    return out if cp == 1 else head_to_seq(out, group)


def split_sequence(x: torch.Tensor, group=None, dim: int = 0) -> torch.Tensor:
    """This rank's contiguous sequence chunk of a full-length tensor (inputs, labels, positions)."""
    group = group if group is not None else dist.group.WORLD
    cp, r = dist.get_world_size(group), dist.get_rank(group)
    assert x.shape[dim] % cp == 0
    return x.chunk(cp, dim=dim)[r].contiguous()
