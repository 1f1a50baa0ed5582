"""Health monitor for the xGMI engines: per-step sticky-error check and a run-wide fallback to RCCL.

Every spin of the xGMI kernels (comm/xgmi.py all-reduce / reduce-scatter / all-gather,
comm/relay.py TP-pair exchange) is bounded: a peer that does not arrive in time makes the waiting
block set a sticky error word in its signal buffer and NaN-fill its output, so the GPU never hangs
(SURVEY §5.3 asks for failure detection instead of the reference's fail-fast-only behaviour,
/root/reference/1_training_mnist_ddp.ipynb:686 ``orte_abort_on_non_zero_status``).

This module turns that word into a recovery, without adding a host-device synchronisation to the
step:

* ``Monitor.launch()`` runs once per training step at a point every rank reaches in the same
  order (``DistributedDataParallel.finish_grad_sync``). On the compute stream it takes the max of
  every live engine's error word (a device tensor aliasing the uncached signal memory) and
  all-reduces it (MAX, world, async); a side stream copies the agreed flag to pinned host memory.
* ``Monitor.consume()`` at the start of the next step (``zero_grad_buffer``) reads that flag,
  waiting for it if needed (the device still has the optimizer of the previous step queued, so it
  does not idle). Every rank sees the same value at the same step and decides identically: a
  tripped flag deactivates every engine (all later collectives take RCCL), logs one warning and
  runs the registered repair callbacks (the optimizer rewrites its parameters from the fp32
  masters and re-gathers the ZeRO shards over RCCL) — before the next forward runs.
* The step that ran on NaN-filled buffers is skipped by the optimizer's device-side found-inf
  check (NaN gradients), so no weight is corrupted. A timeout in a gradient reduction or a TP
  exchange is caught before the next forward (the loss stays finite); one that first hits the
  ZeRO parameter gather after the optimizer shows as one NaN-loss, skipped step.

With no engine on any rank (N = 1, RCCL only, CPU) the monitor costs one world agreement the
first time and nothing after.
"""
from __future__ import annotations

import warnings
import weakref
from typing import Callable, List

import torch
import torch.distributed as dist

_ENGINES: "weakref.WeakSet" = weakref.WeakSet()
_CALLBACKS: List[Callable[[], None]] = []
EVENTS: List[dict] = []          # fallbacks that happened (bench JSON / tests)


def register(engine):
    """An engine with ``error_tensor()`` and ``deactivate(reason)``."""
    _ENGINES.add(engine)


def unregister(engine):
    _ENGINES.discard(engine)


def live_engines():
    return [e for e in list(_ENGINES) if getattr(e, "active", False)]


def on_fallback(cb: Callable[[], None]):
    """Run ``cb()`` after a fallback (a bound method is held weakly)."""
    _CALLBACKS.append(weakref.WeakMethod(cb) if hasattr(cb, "__self__") else (lambda: cb))


class Monitor:
    def __init__(self):
        self.on = None            # world-agreed: does any rank run an engine?
        self.pending = None       # (event or None, pinned flag) of the previous step
        self._stream = None

    def _device(self):
        return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")

    def _host_group(self) -> bool:
        return dist.get_backend() == "gloo"

    def _agree_on(self, dev) -> bool:
        if self.on is None:
            t = torch.tensor([1 if live_engines() else 0], dtype=torch.int32, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            self.on = bool(t.item())
        return self.on

    def _ready(self) -> bool:
        return dist.is_initialized() and dist.get_world_size() > 1 and self.on is not False

    def consume(self):
        """Read the flag launched at the previous gradient sync (blocking until it landed — the
        device still has that step's optimizer queued, so it does not idle) and fall back on every
        rank at once when it is set. Called at the start of each step and before each launch."""
        if self.pending is None:
            return
        ev, pinned = self.pending
        self.pending = None
        if ev is not None:
            ev.synchronize()
        v = int(pinned[0])
        if v:
            self.fallback(v)

    def launch(self):
        """After this step's gradient reduction: max of the live engines' sticky error words,
        all-reduced (MAX) over the world on RCCL's stream, copied to pinned memory by a side
        stream — the compute stream never waits."""
        if not self._ready():
            return
        host = self._host_group()
        dev = torch.device("cpu") if host else self._device()
        if not self._agree_on(dev):
            return
        self.consume()
        if not self.on:
            return
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        for e in live_engines():
            w = e.error_tensor()
            torch.maximum(flag, (w != 0).to(torch.int32).to(dev), out=flag)
        if host:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX)
            self.pending = (None, flag)
            return
        work = dist.all_reduce(flag, op=dist.ReduceOp.MAX, async_op=True)
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=dev)
        pinned = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(self._stream):
            work.wait()                       # the side stream, not the compute stream, waits
            pinned.copy_(flag, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        flag.record_stream(self._stream)
        self.pending = (ev, pinned)

    def fallback(self, code: int = 1):
        """Every rank at once: deactivate the engines, warn, run the repair callbacks."""
        engines = list(_ENGINES)
        names = sorted({type(e).__name__ for e in engines if getattr(e, "active", False)})
        for e in engines:
            try:
                e.deactivate(f"sticky error word {code}")
            except Exception:  # pragma: no cover - best effort
                pass
        EVENTS.append({"error": int(code), "engines": names})
        msg = (f"xGMI engines {names} reported a timed-out peer (error word {code}): the affected step was "
               "skipped (NaN gradients -> found-inf) and every later collective uses RCCL")
        if not dist.is_initialized() or dist.get_rank() == 0:
            warnings.warn(msg, RuntimeWarning)
        for ref in list(_CALLBACKS):
            cb = ref()
            if cb is not None:
                cb()
        self.on = False


_MONITOR = Monitor()


def monitor() -> Monitor:
    return _MONITOR


def reset():
    """Tests: forget engines, callbacks and the world agreement."""
    global _MONITOR
    _ENGINES.clear()
    _CALLBACKS.clear()
    EVENTS.clear()
    _MONITOR = Monitor()
