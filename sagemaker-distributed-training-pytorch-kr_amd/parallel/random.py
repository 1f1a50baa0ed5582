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
    tensor-parallel = default + 2718 + tp_rank."""
    st = ps.get_state()
    s = seed + 100 * st.pp_rank
    if data_parallel_random_init:
        s += 10 * st.dp_rank
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
