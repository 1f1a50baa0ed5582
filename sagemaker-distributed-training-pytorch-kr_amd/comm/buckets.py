"""Gradient-bucket sizing for the 7-link xGMI mesh ("8–32 MB, auto-tuned").

A bucket's collective costs ``t(S) = alpha + S / beta`` on a DP group: ``alpha`` is the launch /
protocol latency, ``beta`` the bus rate the group's links sustain. Small buckets pay ``alpha``
over and over; big ones delay the first reduce-scatter until a large fraction of backward has run
(the first bucket can launch only when ALL its gradients landed), so less of the communication
hides behind backward. The size chosen here is the smallest one at which the latency is at most
10 % of a call (``S = 9 alpha beta``), clamped to [8 MB, 32 MB], and never more than a quarter of
this rank's gradient bytes (at least 4 buckets, so overlap has something to work with).

``alpha`` and ``beta`` come from a short reduce-scatter timing on the real group at two sizes
(collective over the group, ~10 ms at start-up) — the same kind of run-time measurement the xGMI
engine uses to pick its transport. Without a GPU (gloo test groups) a 16 MB nominal size is used.

The reference leaves bucketing to torch DDP's 25 MB default and, for SMDDP, to its
"balanced fusion buffers" (/root/reference/2_training_oxford-pet_ddp.ipynb:387-404).
"""
from __future__ import annotations

import time
from typing import Dict, Optional

import torch
import torch.distributed as dist

MIN_BYTES = 8 << 20
MAX_BYTES = 32 << 20
NOMINAL_BYTES = 16 << 20
MIN_BUCKETS = 4
TUNED: Dict[str, object] = {}          # last decision (bench JSON)


def _time_rs(group, nbytes: int, iters: int = 5) -> float:
    dev = torch.device("cuda", torch.cuda.current_device())
    W = dist.get_world_size(group)
    n = max(W * 64, nbytes // 4 // (W * 64) * (W * 64))
    inp = torch.randn(n, device=dev, dtype=torch.float32)
    out = torch.empty(n // W, device=dev, dtype=torch.float32)
    for _ in range(2):
        dist.reduce_scatter_tensor(out, inp, group=group)
    torch.cuda.synchronize()
    dist.barrier(group=group)
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.reduce_scatter_tensor(out, inp, group=group)
    torch.cuda.synchronize()
    t = torch.tensor([(time.perf_counter() - t0) / iters], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def latency_bandwidth(group, s1: int = 2 << 20, s2: int = 32 << 20):
    """(alpha seconds, beta bytes/s) of reduce-scatter on ``group`` from two timed sizes."""
    t1, t2 = _time_rs(group, s1), _time_rs(group, s2)
    if t2 <= t1:
        return t1, float("inf")
    beta = (s2 - s1) / (t2 - t1)
    alpha = max(0.0, t1 - s1 / beta)
    return alpha, beta


def choose_bucket_bytes(total_bytes: int, alpha: Optional[float] = None, beta: Optional[float] = None) -> int:
    """The bucket size in bytes for ``total_bytes`` of gradients on this rank (see module doc)."""
    if alpha is None or beta is None or beta == float("inf"):
        s = NOMINAL_BYTES
    else:
        s = int(9.0 * alpha * beta)
    s = min(MAX_BYTES, max(MIN_BYTES, s))
    s = min(s, max(1 << 20, total_bytes // MIN_BUCKETS))
    return s


def auto_bucket_elems(group, total_elems: int, elem_bytes: int) -> int:
    """Collective over ``group``: bucket size in ELEMENTS (DDP's unit)."""
    alpha = beta = None
    ws = dist.get_world_size(group) if (dist.is_initialized() and group is not None) else 1
    measured = False
    try:
        rccl = dist.get_backend(group) in ("nccl", "smddp")
    except (RuntimeError, ValueError):     # a group outside c10d's table (comm/loopback.py)
        rccl = False
    if ws > 1 and torch.cuda.is_available() and rccl:
        alpha, beta = latency_bandwidth(group)
        measured = True
    nbytes = choose_bucket_bytes(total_elems * elem_bytes, alpha, beta)
    elems = max(1, nbytes // elem_bytes)
    TUNED.clear()
    TUNED.update({"bucket_MB": round(nbytes / 2 ** 20, 2), "grad_MB": round(total_elems * elem_bytes / 2 ** 20, 1),
                  "source": "measured" if measured else "nominal"})
    if measured:
        TUNED.update({"rs_latency_us": round(alpha * 1e6, 1), "rs_busbw_GBps": round(beta * (ws - 1) / ws / 1e9, 1)})
    return elems
