"""Distributed debugging aids (SURVEY §5.2 / §5.3 — the reference has none; these are the
MI355X build's additions):

* ``CollectiveTracer`` — records (op, shape, dtype, group size) of every torch.distributed
  collective a rank issues and, at ``check()``, all-gathers a rolling hash of that sequence so a
  rank that diverged (a skipped all-reduce, a wrong bucket shape — the classic cause of RCCL
  hangs) is reported by name and step instead of hanging. Enable with
  ``SMDT_COLLECTIVE_CHECK=N`` (check every N steps) or ``CollectiveTracer().install()``.
* ``StepWatchdog`` — if a training step does not finish within ``timeout`` seconds, dumps every
  Python thread's stack (faulthandler) and, optionally, aborts the process so the launcher's
  fail-fast path tears the job down (RCCL collectives that never complete otherwise block
  until the process-group timeout).
* ``maybe_inject_fault(step)`` — deterministic fault injection for tests:
  ``SMDT_FAULT_INJECT="rank=1,step=3,mode=exit|raise|hang|nan|sigterm"``.
* ``enable_async_error_handling()`` — RCCL async error handling / blocking-wait env so a
  collective timeout raises instead of hanging (TORCH_NCCL_ASYNC_ERROR_HANDLING).
"""
from __future__ import annotations

import faulthandler
import hashlib
import os
import signal
import sys
import threading
import time
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

_COLLECTIVES = ("all_reduce", "reduce_scatter_tensor", "all_gather_into_tensor", "broadcast", "all_gather",
                "reduce_scatter", "all_to_all_single", "barrier", "reduce")


def enable_async_error_handling(blocking_wait: bool = False):
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if blocking_wait:
        os.environ.setdefault("TORCH_NCCL_BLOCKING_WAIT", "1")


class CollectiveTracer:
    """Wraps ``torch.distributed`` collectives to fingerprint the per-rank call sequence."""

    def __init__(self, keep: int = 64, log_path: Optional[str] = None):
        self.records: List[Tuple[str, tuple, str, int]] = []
        # every call as issued, one line each, flushed at once (a hang leaves the per-rank
        # sequences on disk to compare: SMDT_COLLECTIVE_LOG=<prefix> writes <prefix>.rank<R>)
        self._log = open(log_path, "w", buffering=1) if log_path else None
        self.digest = hashlib.sha1()
        self.count = 0
        self.keep = keep
        self._orig = {}
        self.step = 0

    def _wrap(self, name, fn):
        tracer = self

        def wrapped(*args, **kwargs):
            t = args[0] if args and isinstance(args[0], torch.Tensor) else kwargs.get("tensor")
            if t is None and args and isinstance(args[0], (list, tuple)) and args[0] and \
                    isinstance(args[0][0], torch.Tensor):
                t = args[0][0]
            group = kwargs.get("group")
            gsz = dist.get_world_size(group) if dist.is_initialized() else 1
            rec = (name, tuple(t.shape) if t is not None else (), str(t.dtype) if t is not None else "", gsz)
            tracer.digest.update(repr(rec).encode())
            tracer.count += 1
            if tracer._log is not None:
                tracer._log.write(f"{tracer.count} {time.time():.6f} {rec} async={kwargs.get('async_op', False)}\n")
            tracer.records.append(rec)
            if len(tracer.records) > tracer.keep:
                tracer.records.pop(0)
            return fn(*args, **kwargs)

        wrapped._smdt_traced = True
        return wrapped

    def install(self):
        for n in _COLLECTIVES:
            fn = getattr(dist, n, None)
            if fn is not None and not getattr(fn, "_smdt_traced", False):
                self._orig[n] = fn
                setattr(dist, n, self._wrap(n, fn))
        return self

    def uninstall(self):
        for n, fn in self._orig.items():
            setattr(dist, n, fn)
        self._orig.clear()

    def check(self, group=None) -> Optional[str]:
        """All-gather (count, digest) over ``group``; returns None when every rank agrees, else a
        human-readable report (also printed) naming the diverging ranks and their last ops."""
        self.step += 1
        if not dist.is_initialized() or dist.get_world_size(group) == 1:
            return None
        fn = self._orig.get("all_gather_object", dist.all_gather_object)
        mine = (self.count, self.digest.hexdigest()[:16], self.records[-4:])
        ws = dist.get_world_size(group)
        allv = [None] * ws
        # all_gather_object is not wrapped, so the check itself does not perturb the digest
        fn(allv, mine, group=group)
        sigs = {(c, d) for c, d, _ in allv}
        if len(sigs) == 1:
            return None
        lines = [f"[smdt collective-check] step {self.step}: ranks disagree on the collective sequence"]
        for r, (c, d, last) in enumerate(allv):
            lines.append(f"  rank {r}: {c} collectives, digest {d}, last {last}")
        msg = "\n".join(lines)
        print(msg, file=sys.stderr, flush=True)
        return msg


_TRACER: Optional[CollectiveTracer] = None


def collective_log_from_env():
    """SMDT_COLLECTIVE_LOG=<prefix>: trace every collective of this rank into <prefix>.rank<R>
    (installed once; returns the tracer or None)."""
    global _TRACER
    pre = os.environ.get("SMDT_COLLECTIVE_LOG")
    if not pre or _TRACER is not None:
        return _TRACER
    r = dist.get_rank() if dist.is_initialized() else 0
    _TRACER = CollectiveTracer(log_path=f"{pre}.rank{r}").install()
    return _TRACER


def collective_check_from_env(step: int, group=None):
    """Hook for training loops: installs the tracer on first call when SMDT_COLLECTIVE_CHECK is
    set and checks every N steps; raises on divergence."""
    global _TRACER
    n = int(os.environ.get("SMDT_COLLECTIVE_CHECK", "0") or 0)
    if n <= 0:
        return
    if _TRACER is None:
        _TRACER = CollectiveTracer().install()
        return
    if step % n == 0:
        msg = _TRACER.check(group)
        if msg:
            raise RuntimeError(msg)


class StepWatchdog:
    """``with StepWatchdog(600): train_step()`` — stack dump (and abort) if the step hangs."""

    def __init__(self, timeout: float, abort: bool = True, file=None):
        self.timeout = float(timeout)
        self.abort = abort
        self.file = file or sys.stderr
        self._timer: Optional[threading.Timer] = None

    def _fire(self):
        print(f"[smdt watchdog] step exceeded {self.timeout:.0f}s on rank "
              f"{dist.get_rank() if dist.is_initialized() else 0}; dumping stacks", file=self.file, flush=True)
        faulthandler.dump_traceback(file=self.file, all_threads=True)
        if self.abort:
            os.kill(os.getpid(), signal.SIGABRT)

    def __enter__(self):
        if self.timeout > 0:
            self._timer = threading.Timer(self.timeout, self._fire)
            self._timer.daemon = True
            self._timer.start()
        return self

    def __exit__(self, *exc):
        if self._timer is not None:
            self._timer.cancel()
        return False


def parse_fault_spec(spec: str):
    out = {"rank": None, "step": None, "mode": "exit"}
    for part in filter(None, (p.strip() for p in spec.split(","))):
        k, _, v = part.partition("=")
        out[k.strip()] = v.strip()
    if out["rank"] is not None:
        out["rank"] = int(out["rank"])
    if out["step"] is not None:
        out["step"] = int(out["step"])
    return out


def maybe_inject_fault(step: int, rank: Optional[int] = None, loss: Optional[torch.Tensor] = None):
    """Deterministic fault injection driven by ``SMDT_FAULT_INJECT`` (tests / chaos runs).
    Modes: exit (os._exit(13)), raise (RuntimeError), hang (sleep forever), sigterm (signal to
    self, exercising --exit-signal-handler), nan (poison ``loss`` in place)."""
    spec = os.environ.get("SMDT_FAULT_INJECT")
    if not spec:
        return
    f = parse_fault_spec(spec)
    if rank is None:
        rank = dist.get_rank() if dist.is_initialized() else int(os.environ.get("RANK", "0"))
    if (f["rank"] is not None and f["rank"] != rank) or (f["step"] is not None and f["step"] != step):
        return
    mode = f["mode"]
    print(f"[smdt fault-inject] rank {rank} step {step}: {mode}", file=sys.stderr, flush=True)
    if mode == "exit":
        os._exit(13)
    elif mode == "raise":
        raise RuntimeError(f"injected fault at step {step} on rank {rank}")
    elif mode == "hang":
        while True:
            time.sleep(3600)
    elif mode == "sigterm":
        os.kill(os.getpid(), signal.SIGTERM)
    elif mode == "nan" and loss is not None:
        with torch.no_grad():
            loss.fill_(float("nan"))
