"""Parallel-aware RNG and activation recompute.

Megatron keeps two RNG streams (SURVEY P9 / `--seed` at
/root/reference/3_training_megatron-lm/megatron/arguments.py:861-863): a *default* stream that
is identical across tensor-parallel ranks (dropout on replicated activations must agree) and a
*model-parallel* stream that differs per TP rank (dropout on sharded activations). Our fused
dropout kernels are counter-based (Philox, keyed by (seed, offset, element)), so each stream is
just a (seed, offset) pair; recompute replays a region by rewinding the offsets.
"""
from __future__ import annotations

import contextlib
import random as _pyrandom

import numpy as np
import torch
import torch.utils.checkpoint as tcp

from ..ops.functional import PhiloxState
from ..ops import functional as SF
from . import state as ps

_TRACKERS = {"default": SF.default_rng(), "tp": PhiloxState(1234 + 2718)}


def get_rng(kind: str = "default") -> PhiloxState:
    return _TRACKERS[kind]


def model_parallel_seed(seed: int, data_parallel_random_init: bool = False):
    """Seed torch / numpy / python and both Philox streams, Megatron-style:
    default = seed + 100 * pp_rank (+ 10 * dp_rank with data-parallel random init),
    tensor-parallel = default + 2718 + tp_rank. Context-parallel ranks see different tokens (and,
    inside Ulysses attention, different heads), so cp_rank > 0 shifts both streams by 7919 * cp_rank
    (cp = 1 leaves every seed unchanged)."""
    st = ps.get_state()
    s = seed + 100 * st.pp_rank
    if data_parallel_random_init:
        s += 10 * st.dp_rank
    if getattr(st, "cp", 1) > 1:
        s += 7919 * st.cp_rank
    _pyrandom.seed(s)
    np.random.seed(s % (2 ** 32))
    torch.manual_seed(s)
    _TRACKERS["default"].seed, _TRACKERS["default"].offset = s, 0
    _TRACKERS["tp"].seed, _TRACKERS["tp"].offset = s + 2718 + st.tp_rank, 0
    return s


def rng_state_dict():
    d = {k: v.state_dict() for k, v in _TRACKERS.items()}
    d["torch_cpu"] = torch.get_rng_state()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        d["torch_cuda"] = torch.cuda.get_rng_state()
    d["numpy"] = np.random.get_state()
    d["python"] = _pyrandom.getstate()
    return d


def load_rng_state_dict(d):
    for k, v in _TRACKERS.items():
        if k in d:
            v.load_state_dict(d[k])
    if "torch_cpu" in d:
        torch.set_rng_state(d["torch_cpu"])
    if "torch_cuda" in d and torch.cuda.is_available():
        torch.cuda.set_rng_state(d["torch_cuda"])
    if "numpy" in d:
        np.random.set_state(d["numpy"])
    if "python" in d:
        _pyrandom.setstate(d["python"])


def _philox_context_fn():
    saved = {k: v.offset for k, v in _TRACKERS.items()}

    @contextlib.contextmanager
    def forward_ctx():
        yield

    @contextlib.contextmanager
    def recompute_ctx():
        now = {k: v.offset for k, v in _TRACKERS.items()}
        for k, v in _TRACKERS.items():
            v.offset = saved[k]
        try:
            yield
        finally:
            for k, v in _TRACKERS.items():
                v.offset = now[k]

    return forward_ctx(), recompute_ctx()


def checkpoint(fn, *args):
    """Activation recompute (``--recompute-granularity full``) that replays dropout masks
    exactly: torch RNG via ``preserve_rng_state`` and the Philox streams via offset rewind."""
    return tcp.checkpoint(fn, *args, use_reentrant=False, preserve_rng_state=True, context_fn=_philox_context_fn)


class _DistributedCheckpoint(torch.autograd.Function):
    """Full-layer recompute whose saved layer input is split across the tensor-parallel ranks
    (Megatron ``--distribute-saved-activations``, /root/reference/3_training_megatron-lm/megatron/
    arguments.py:746-760): each TP rank keeps 1/tp of the (TP-replicated) input between forward and
    backward and the slices are all-gathered right before the recompute. Dropout masks replay
    exactly (torch RNG state + Philox offsets restored)."""

    @staticmethod
    def forward(ctx, run_fn, nargs, *args):
        from . import state as ps
        import torch.distributed as dist
        st = ps.get_state()
        ctx.run_fn = run_fn
        ctx.cpu_state = torch.get_rng_state()
        ctx.cuda_state = torch.cuda.get_rng_state() if (torch.cuda.is_available() and torch.cuda.is_initialized()) \
            else None
        ctx.philox = {k: v.offset for k, v in _TRACKERS.items()}
        with torch.no_grad():
            out = run_fn(*args)
        # fresh aliases: a parameter returned as-is (the pending fc2 bias) must not become an
        # output of this node; its gradient is routed through the recompute in backward
        if isinstance(out, tuple):
            out = tuple(o.detach() if isinstance(o, torch.Tensor) else o for o in out)
        elif isinstance(out, torch.Tensor):
            out = out.detach()
        x = args[0]
        ctx.x_shape = x.shape
        ctx.tp = st.tp if (st.tp > 1 and st.tp_group is not None) else 1
        keep = x
        if ctx.tp > 1:
            flat = x.detach().contiguous().view(-1)
            assert flat.numel() % ctx.tp == 0, "distribute-saved-activations: input numel must divide tp"
            keep = flat.chunk(ctx.tp)[st.tp_rank].clone()
        ctx.arg_is_tensor = [isinstance(a, torch.Tensor) for a in args]
        ctx.others = [None if isinstance(a, torch.Tensor) else a for a in args]
        ctx.save_for_backward(keep, *[a for a in args[1:] if isinstance(a, torch.Tensor)])
        return out

    @staticmethod
    def backward(ctx, *grads):
        from . import state as ps
        import torch.distributed as dist
        st = ps.get_state()
        keep, *rest = ctx.saved_tensors
        if ctx.tp > 1:
            full = torch.empty(keep.numel() * ctx.tp, dtype=keep.dtype, device=keep.device)
            dist.all_gather_into_tensor(full, keep, group=st.tp_group)
            x = full.view(ctx.x_shape)
        else:
            x = keep
        it = iter(rest)
        args = []
        for i, is_t in enumerate(ctx.arg_is_tensor):
            a = (x if i == 0 else next(it)) if is_t else ctx.others[i]
            if isinstance(a, torch.Tensor):
                a = a.detach().requires_grad_(a.is_floating_point())
            args.append(a)
        now_cpu = torch.get_rng_state()
        now_cuda = torch.cuda.get_rng_state() if ctx.cuda_state is not None else None
        now_philox = {k: v.offset for k, v in _TRACKERS.items()}
        torch.set_rng_state(ctx.cpu_state)
        if ctx.cuda_state is not None:
            torch.cuda.set_rng_state(ctx.cuda_state)
        for k, v in _TRACKERS.items():
            v.offset = ctx.philox[k]
        try:
            with torch.enable_grad():
                out = ctx.run_fn(*args)
        finally:
            torch.set_rng_state(now_cpu)
            if now_cuda is not None:
                torch.cuda.set_rng_state(now_cuda)
            for k, v in _TRACKERS.items():
                v.offset = now_philox[k]
        outs = out if isinstance(out, tuple) else (out,)
        pairs = [(o, g) for o, g in zip(outs, grads) if isinstance(o, torch.Tensor) and o.requires_grad
                 and g is not None]
        torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None) + tuple(a.grad if isinstance(a, torch.Tensor) else None for a in args)


def distributed_checkpoint(fn, *args):
    """``checkpoint`` with the first argument's saved copy split across the TP group."""
    return _DistributedCheckpoint.apply(fn, len(args), *args)
