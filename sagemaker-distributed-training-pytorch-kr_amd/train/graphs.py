"""Whole-training-step HIP graphs.

An eager image-model step issues 1.5-3.7 k kernel launches; with the host launching them one by
one the device idles 5-42 ms per step (profiles/r4_vision/). ``CapturedStep`` runs a step
function eagerly for a few warm-up calls (MIOpen / hipBLASLt algorithm selection, lazily built
buffers), captures one call in a HIP graph and replays it from then on: the inputs are copied
into the graph's static buffers and the step's outputs are the graph's static tensors.

What may be inside the step: the forward / backward, the framework DDP's bucketed gradient
reductions (RCCL collectives and the loopback stand-ins of rank emulation are captured; the xGMI
IPC engine sits out a capture, ``DistributedDataParallel._xg``) and an optimizer whose step count
lives on the device (``MixedPrecisionAdam(capturable=True)``, torch's ``capturable=True`` Adam).
Nothing in the step may synchronise with the host. A call whose inputs do not match the captured
shapes (a short last batch) runs eagerly on the same model / optimizer state.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch


class CapturedStep:
    def __init__(self, fn: Callable, warmup: int = 2, enabled: bool = True):
        self.fn = fn
        self.warmup = int(warmup)
        self.enabled = bool(enabled) and torch.cuda.is_available()
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_in: Sequence[torch.Tensor] = ()
        self.static_out = None
        self.note = "eager" if not self.enabled else "warming up"

    def _matches(self, inputs) -> bool:
        return (len(inputs) == len(self.static_in)
                and all(a.shape == b.shape and a.dtype == b.dtype and a.device == b.device
                        for a, b in zip(inputs, self.static_in)))

    def __call__(self, *inputs: torch.Tensor):
        self.calls += 1
        if not self.enabled or self.calls <= self.warmup or not all(t.is_cuda for t in inputs):
            return self.fn(*inputs)
        if self.graph is None:
            try:
                self.static_in = [t.detach().clone() for t in inputs]
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.static_out = self.fn(*self.static_in)
                self.graph = g
                self.note = "captured"
            except Exception as e:  # noqa: BLE001 - report and stay eager
                self.enabled = False
                self.graph = None
                self.note = f"capture failed, eager: {type(e).__name__}: {str(e)[:160]}"
                torch.cuda.synchronize()
                return self.fn(*inputs)
            # the capture ran no kernels: this call's step still has to happen
        elif not self._matches(inputs):
            return self.fn(*inputs)
        for s, t in zip(self.static_in, inputs):
            s.copy_(t, non_blocking=True)
        self.graph.replay()
        return self.static_out
