"""Per-step phase timing and per-collective accounting (SURVEY §5.5 "per-collective bus-bandwidth").

The reference's only view of its communication is NCCL's topology / channel log
(/root/reference/1_training_mnist_ddp.ipynb:936-977, 3_training_megatron-lm.ipynb:1440-1452); a
slow multi-GPU step cannot be explained from its output. This module makes a training step
explain itself:

* **phases** — CUDA events recorded on the compute stream at the step's boundaries (start,
  forward/backward done, gradient sync done, optimizer done) split the step's GPU time into
  forward/backward, DP gradient sync and optimizer. Inside forward/backward, every place where the
  compute stream WAITS for communication (a TP ring exchange, a pipeline receive, a ZeRO parameter
  gather, a blocking TP all-reduce) is bracketed by an event pair on the same stream: the stall
  is attributed to its axis (tp / pp / dp / cp) and the remainder is compute. The pieces sum to
  the step's device time by construction; the host gap between steps is reported separately.
* **collectives** — every collective the framework issues is counted with its axis, op, bytes and
  transport (RCCL, the xGMI IPC kernel, the TP-pair relay) and timed: RCCL works through
  ``TORCH_NCCL_ENABLE_TIMING`` (start / end events on RCCL's own stream), the xGMI engines through
  start / end events on their side stream, blocking calls through the event pair around them.
  Bus bandwidth uses the nccl-tests conventions (all-reduce 2(n-1)/n, reduce-scatter /
  all-gather / all-to-all (n-1)/n, p2p 1).

Off by default (no cost). ``enable()`` before the process group exists (it sets
``TORCH_NCCL_ENABLE_TIMING``); ``begin_step()`` / ``mark()`` / ``end_step()`` around each step;
``summary()`` averages per step. On CPU (gloo) host timestamps replace the events, so the same
accounting runs in the multi-process tests. Timings are read only once the device has finished a
step (non-blocking checks at later step ends), so the timed loop is never synchronised.
"""
from __future__ import annotations

import contextlib
import os
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

_ON = False
_CUDA = False
_STEP = None
_DEPTH = [0]                      # nested waits are counted once (the outermost)
_POOL: List = []                  # recycled timing events
_UNRESOLVED: List = []            # closed steps the device may still be running
_PENDING: List = []               # (coll record, in-flight work)
_TOT: Dict = {}

BUS_FACTOR = {
    "all_reduce": lambda n: 2.0 * (n - 1) / n,
    "reduce_scatter": lambda n: (n - 1) / n,
    "all_gather": lambda n: (n - 1) / n,
    "all_to_all": lambda n: (n - 1) / n,
    "broadcast": lambda n: 1.0,
    "p2p": lambda n: 1.0,
}


def enable(on: bool = True, cuda: Optional[bool] = None):
    """Turn accounting on (call before ``init_process_group`` so RCCL records per-work timings)."""
    global _ON, _CUDA
    _ON = bool(on)
    _CUDA = torch.cuda.is_available() if cuda is None else bool(cuda)
    if _ON and _CUDA:
        os.environ.setdefault("TORCH_NCCL_ENABLE_TIMING", "1")
    reset()


def active() -> bool:
    return _ON and _STEP is not None


def reset():
    global _STEP
    _STEP = None
    _UNRESOLVED.clear()
    _PENDING.clear()
    _TOT.clear()
    _TOT.update(steps=0, phase=defaultdict(float), host_gap=0.0, gaps=0, device=0.0, coll={}, prev_end=None)


reset()


def _stamp():
    if _CUDA:
        ev = _POOL.pop() if _POOL else torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev
    return time.perf_counter()


def _ms(a, b) -> float:
    if _CUDA:
        return float(a.elapsed_time(b))
    return (b - a) * 1e3


def axis_of(group) -> str:
    from ..parallel import state as ps
    st = ps.get_state() if ps.model_parallel_is_initialized() else None
    if st is not None:
        for name, g in (("tp", st.tp_group), ("pp", st.pp_group), ("dp", st.dp_group),
                        ("dp", st.dp_cp_group), ("cp", st.cp_group), ("embd", st.embd_group),
                        ("mp", st.mp_group)):
            if g is not None and group is g:
                return name
    return "world"


def _size(group) -> int:
    try:
        return dist.get_world_size(group)
    except (RuntimeError, ValueError):
        return 1


class _Step:
    __slots__ = ("marks", "waits", "colls")

    def __init__(self):
        self.marks: List[tuple] = []
        self.waits: List[tuple] = []
        # [axis, op, bytes, ranks, transport, ms, events, shared, work still in flight]
        self.colls: List[list] = []


def begin_step():
    global _STEP
    if not _ON:
        return
    _STEP = _Step()
    _STEP.marks.append(("start", _stamp()))


def mark(name: str):
    """Close the phase that ends here (names: 'fwd_bwd', 'grad_sync', 'optimizer')."""
    if _ON and _STEP is not None:
        _STEP.marks.append((name, _stamp()))


@contextlib.contextmanager
def waiting(axis: str):
    """Bracket a point where the compute stream waits for communication on ``axis``."""
    if not (_ON and _STEP is not None) or _DEPTH[0]:
        yield
        return
    _DEPTH[0] += 1
    a = _stamp()
    try:
        yield
    finally:
        _DEPTH[0] -= 1
        _STEP.waits.append((axis, a, _stamp()))


def _backend_label(group) -> str:
    """The library behind ``group``'s collectives: rccl (nccl / smddp on GPU) or gloo."""
    try:
        import torch.distributed as dist
        return "gloo" if dist.get_backend(group) == "gloo" else "rccl"
    except (RuntimeError, ValueError):
        return "rccl"


def collective(op: str, group, nbytes: int, work=None, transport: str = "rccl", events=None):
    """Count an issued collective. ``work``: an async torch work (its RCCL timing is read once it
    completed); ``events``: (start, end) events of an xGMI engine call. ``nbytes``: see
    BUS_FACTOR's ops (all-reduce: tensor; reduce-scatter: input; all-gather: output; p2p: sent)."""
    if not (_ON and _STEP is not None):
        return
    has_work = work is not None and _CUDA
    if transport == "rccl":
        transport = _backend_label(group)
    rec = [axis_of(group), op, int(nbytes), _size(group), transport, None, events, None, has_work]
    _STEP.colls.append(rec)
    if has_work:
        # A work keeps its tensors alive: hold it only while it is in flight (polled, so at most
        # the collectives the host is ahead of the device by stay referenced).
        _PENDING.append((rec, work))
        if len(_PENDING) > 32:
            _poll(_PENDING)


def _poll(pending, force: bool = False):
    keep = []
    for rec, work in pending:
        try:
            done = force or work.is_completed()
        except Exception:
            done = True
        if done:
            rec[5] = _work_ms(work)
            rec[8] = False
        else:
            keep.append((rec, work))
    pending[:] = keep


@contextlib.contextmanager
def blocking(op: str, group, nbytes: int, transport: str = "rccl", axis: Optional[str] = None):
    """A collective whose completion the compute stream waits for right away: it is a wait on
    its axis AND a timed collective (its duration is the bracketed interval)."""
    if not (_ON and _STEP is not None) or _DEPTH[0]:
        yield
        return
    ax = axis or axis_of(group)
    _DEPTH[0] += 1
    a = _stamp()
    try:
        yield
    finally:
        _DEPTH[0] -= 1
        b = _stamp()
        _STEP.waits.append((ax, a, b))
        if transport == "rccl":
            transport = _backend_label(group)
        _STEP.colls.append([ax, op, int(nbytes), _size(group), transport, None, (a, b), "shared", False])


def _work_ms(work) -> Optional[float]:
    if work is None:
        return None
    try:
        d = work._get_duration()
        return float(d) if d is not None and d >= 0 else None
    except Exception:  # gloo works / timing off: bytes are still counted
        return None


def end_step():
    """Close the step. Its timings are resolved once the device has finished it (checked without
    blocking at later step ends; ``flush`` / ``summary`` wait for the rest), so collecting stats
    adds no host-device synchronisation to the timed loop."""
    global _STEP
    if not (_ON and _STEP is not None):
        return
    _STEP.marks.append(("end", _stamp()))
    _UNRESOLVED.append(_STEP)
    _STEP = None
    _resolve(block=False)


def flush():
    """Wait for the device and resolve every closed step."""
    if _CUDA:
        torch.cuda.synchronize()
    _resolve(block=True)


def _done(step) -> bool:
    if not _CUDA:
        return True
    return step.marks[-1][1].query()


def _resolve(block: bool):
    _poll(_PENDING, force=block)
    while _UNRESOLVED and (block or (_done(_UNRESOLVED[0]) and not any(r[5] is None and r[8]
                                                                      for r in _UNRESOLVED[0].colls))):
        _account(_UNRESOLVED.pop(0))


def _account(s):
    t0 = s.marks[0][1]
    pos = {}
    prev = t0
    for name, ev in s.marks[1:]:
        pos[name] = (_ms(t0, prev), _ms(t0, ev))
        if name != "end":
            _TOT["phase"][name] += _ms(prev, ev)
        prev = ev
    device_ms = _ms(t0, s.marks[-1][1])
    fb_end = pos.get("fwd_bwd", (0.0, device_ms))[1]
    for axis, a, b in s.waits:
        where = "fwd_bwd" if _ms(t0, a) < fb_end else "late"
        _TOT["phase"][f"wait:{axis}:{where}"] += _ms(a, b)
    for axis, op, nb, n, transport, ms, evs, shared, _has_work in s.colls:
        if evs is not None:
            ms = _ms(evs[0], evs[1])
        key = (axis, op, transport)
        c = _TOT["coll"].setdefault(key, {"calls": 0, "bytes": 0, "bus_bytes": 0.0, "ms": 0.0, "world": n})
        c["calls"] += 1
        c["bytes"] += nb
        if ms is not None and ms > 0:
            c["ms"] += ms
            c["bus_bytes"] += nb * BUS_FACTOR.get(op, lambda _n: 1.0)(max(n, 2))
    _TOT["device"] += device_ms
    if _TOT["prev_end"] is not None:     # device idle between the previous step and this one
        _TOT["host_gap"] += max(0.0, _ms(_TOT["prev_end"], t0))
        _TOT["gaps"] += 1
    _TOT["steps"] += 1
    if _CUDA:
        if _TOT["prev_end"] is not None:
            _POOL.append(_TOT["prev_end"])
        _POOL.extend(ev for name, ev in s.marks[:-1])
        for _, a, b in s.waits:
            _POOL.extend((a, b))
        # engine events (colls without "shared") belong to handles that may still be waited on
    _TOT["prev_end"] = s.marks[-1][1]


def summary(ms_per_step: Optional[float] = None) -> Dict[str, dict]:
    """Per-step means: ``phase_ms`` (sums to the step time) and ``comm`` (per axis and op)."""
    flush()
    n = max(1, _TOT["steps"])
    ph = _TOT["phase"]
    fb = ph.get("fwd_bwd", 0.0)
    waits = {k: v for k, v in ph.items() if k.startswith("wait:")}
    fb_waits = defaultdict(float)
    for k, v in waits.items():
        _, axis, where = k.split(":")
        if where == "fwd_bwd":
            fb_waits[axis] += v
    out = {
        "fwd_bwd_compute": (fb - sum(fb_waits.values())) / n,
        "tp_exchange_wait": (fb_waits.get("tp", 0.0) + fb_waits.get("cp", 0.0)) / n,
        "pp_p2p_wait_and_bubble": fb_waits.get("pp", 0.0) / n,
        "dp_param_gather_wait": fb_waits.get("dp", 0.0) / n,
        "other_comm_wait": sum(v for a, v in fb_waits.items() if a not in ("tp", "cp", "pp", "dp")) / n,
        "dp_grad_sync": ph.get("grad_sync", 0.0) / n,
        "optimizer": ph.get("optimizer", 0.0) / n,
        "host_gap": _TOT["host_gap"] / max(1, _TOT["gaps"]),
    }
    phase = {k: round(v, 3) for k, v in out.items()}
    phase["sum"] = round(sum(out.values()), 3)
    if ms_per_step is not None:
        phase["ms_per_step"] = round(ms_per_step, 3)
    comm: Dict[str, dict] = {}
    for (axis, op, transport), c in sorted(_TOT["coll"].items()):
        a = comm.setdefault(axis, {"calls": 0, "MB": 0.0, "ms": 0.0, "ops": {}})
        a["calls"] += c["calls"] / n
        a["MB"] += c["bytes"] / n / 1e6
        a["ms"] += c["ms"] / n
        a["ops"][f"{op}/{transport}"] = {
            "calls": round(c["calls"] / n, 2), "MB": round(c["bytes"] / n / 1e6, 3),
            "ms": round(c["ms"] / n, 3), "ranks": c["world"],
            "busbw_GBps": round(c["bus_bytes"] / (c["ms"] * 1e6), 2) if c["ms"] > 0 else None,
        }
    for a in comm.values():
        a["calls"] = round(a["calls"], 2)
        a["MB"] = round(a["MB"], 3)
        a["ms"] = round(a["ms"], 3)
    return {"phase_ms": phase, "comm": comm, "steps": _TOT["steps"]}
