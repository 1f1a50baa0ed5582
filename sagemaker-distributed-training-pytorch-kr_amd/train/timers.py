"""Megatron-format named timers.

``timers('batch-generator', log_level=2).start()/.stop()`` (reference `pretrain_gpt.py:109-112`),
``--timing-log-level 0..2``, ``--timing-log-option max|minmax|all``,
``--no-barrier-with-level-1-timing`` (/root/reference/3_training_megatron-lm/megatron/
arguments.py:626-651); output block "(min, max) time across ranks (ms):" (NB3:3164).

Timers synchronise the device before reading the clock (``torch.cuda.synchronize``) only when
they are active at the configured log level, so level-2 timers cost nothing by default.
Optional roctx ranges make the same names visible in rocprofv3 traces.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

try:  # roctx markers for rocprofv3 --marker-trace (optional)
    import ctypes
    _roctx = ctypes.CDLL("libroctx64.so")
    _roctx.roctxRangePushA.argtypes = [ctypes.c_char_p]
except Exception:  # pragma: no cover
    _roctx = None


def _sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


class _Timer:
    def __init__(self, name: str, roctx: bool = False):
        self.name = name
        self.elapsed_ = 0.0
        self.started = False
        self.start_time = 0.0
        self.roctx = roctx and _roctx is not None

    def start(self, barrier=False):
        assert not self.started, f"timer {self.name} has already been started"
        if barrier and dist.is_initialized():
            dist.barrier()
        _sync()
        if self.roctx:
            _roctx.roctxRangePushA(self.name.encode())
        self.start_time = time.time()
        self.started = True

    def stop(self, barrier=False):
        assert self.started, f"timer {self.name} is not started"
        if barrier and dist.is_initialized():
            dist.barrier()
        _sync()
        self.elapsed_ += time.time() - self.start_time
        if self.roctx:
            _roctx.roctxRangePop()
        self.started = False

    def reset(self):
        self.elapsed_ = 0.0
        self.started = False

    def elapsed(self, reset=True, barrier=False):
        was = self.started
        if was:
            self.stop(barrier)
        e = self.elapsed_
        if reset:
            self.reset()
        if was:
            self.start(barrier)
        return e


class _DummyTimer:
    def start(self, barrier=False):
        pass

    def stop(self, barrier=False):
        pass

    def elapsed(self, reset=True, barrier=False):
        raise RuntimeError("dummy timer should not be used to calculate elapsed time")


class Timers:
    def __init__(self, log_level: int = 0, log_option: str = "minmax", roctx: bool = False):
        self.log_level = log_level
        self.log_option = log_option
        self.roctx = roctx
        self._timers: Dict[str, _Timer] = {}
        self._levels: Dict[str, int] = {}
        self._dummy = _DummyTimer()
        self._max_level = 2

    def __call__(self, name, log_level=None):
        if name in self._timers:
            if log_level is not None:
                assert log_level == self._levels[name]
            return self._timers[name]
        if log_level is None:
            log_level = self._max_level
        if log_level > self.log_level:
            return self._dummy
        self._timers[name] = _Timer(name, self.roctx)
        self._levels[name] = log_level
        return self._timers[name]

    def _gather(self, names, reset, barrier):
        if barrier and dist.is_initialized():
            dist.barrier()
        ws = dist.get_world_size() if dist.is_initialized() else 1
        rk = dist.get_rank() if dist.is_initialized() else 0
        dev = torch.device("cuda", torch.cuda.current_device()) if (torch.cuda.is_available() and dist.is_initialized() and dist.get_backend() in ("nccl", "smddp")) else torch.device("cpu")
        t = torch.zeros(ws, len(names), dtype=torch.float, device=dev)
        for i, n in enumerate(names):
            if n in self._timers:
                t[rk, i] = self._timers[n].elapsed(reset=reset)
        if dist.is_initialized() and ws > 1:
            out = torch.zeros_like(t)
            dist.all_reduce(t)  # each rank filled only its own row
            out = t
            t = out
        return t.cpu()

    def get_all_timers_string(self, names: Optional[List[str]] = None, normalizer=1.0, reset=True, barrier=False):
        names = [n for n in (names or list(self._timers)) if n in self._timers]
        if not names:
            return None
        t = self._gather(names, reset, barrier) * 1000.0 / normalizer
        if self.log_option == "max":
            s = "max time across ranks (ms):"
            for i, n in enumerate(names):
                s += f"\n    {n} {'.' * max(1, 40 - len(n))}: {t[:, i].max().item():.2f}"
        elif self.log_option == "minmax":
            s = "(min, max) time across ranks (ms):"
            for i, n in enumerate(names):
                s += f"\n    {n} {'.' * max(1, 40 - len(n))}: ({t[:, i].min().item():.2f}, {t[:, i].max().item():.2f})"
        else:
            s = "times across ranks (ms):"
            for i, n in enumerate(names):
                s += f"\n  {n}:" + "".join(f"\n     rank {r:2d}: {t[r, i].item():.2f}" for r in range(t.shape[0]))
        return s

    def log(self, names=None, normalizer=1.0, reset=True, barrier=False):
        s = self.get_all_timers_string(names, normalizer, reset, barrier)
        last = (not dist.is_initialized()) or dist.get_rank() == dist.get_world_size() - 1
        if s is not None and last:
            print(s, flush=True)

    def write(self, names, writer, iteration, normalizer=1.0, reset=False, barrier=False):
        """Megatron's ``Timers.write``: max-over-ranks time of each timer as ``<name>-time``
        scalars (collective: every rank calls it; only ranks with a writer write)."""
        names = [n for n in names if n in self._timers]
        if not names:
            return
        t = self._gather(names, reset, barrier) / normalizer
        if writer is not None:
            for i, n in enumerate(names):
                writer.add_scalar(f"{n}-time", t[:, i].max().item(), iteration)
