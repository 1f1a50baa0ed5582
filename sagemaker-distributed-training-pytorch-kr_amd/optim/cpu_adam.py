"""ZeRO optimizer offload: AdamW state in pinned host memory, updated by the native
``_runtime.cpu_adam`` kernel (DeepSpeed ``offload_optimizer: {device: cpu}`` — SURVEY P8;
/root/reference/4_training_alpaca_deepspeed/configs/default_offload_opt_param-original.json:24-28).

Per step: grad-norm/inf check on the device (HIP sumsq over this rank's shard, all-reduced) ->
one host sync for the clip coefficient -> per piece: D2H of the reduced fp32 grad shard into a
pinned buffer, host AdamW writing fp32 master + a bf16 copy, H2D of the bf16 copy into the flat
param buffer -> ZeRO all-gather. D2H of piece i+1 overlaps the host update of piece i.

On MI355X this is only useful for models whose fp32 optimizer state exceeds HBM (> ~20 B params
per GPU with ZeRO over 8); it exists for config parity.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from ..parallel import tensor_parallel as _tp
from .optimizer import MixedPrecisionAdam


class CPUOffloadAdam(MixedPrecisionAdam):
    def __init__(self, ddp, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, adamw=True, clip_grad=0.0,
                 loss_scaler=None, use_distributed_optimizer: Optional[bool] = None, threads: int = 0):
        from .. import _runtime
        self._rt = _runtime
        self.threads = threads
        self.ddp = ddp
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.adamw = adamw
        self.clip_grad = clip_grad
        self.zero = ddp.zero if use_distributed_optimizer is None else use_distributed_optimizer
        self.scaler = loss_scaler
        self.step_count = 0
        self.device = ddp.grad_data.device
        self.pieces = []
        if self.zero:
            for b in ddp.buckets:
                s, e = ddp.shard_range(b)
                self.pieces.append((s, e, b.region))
        else:
            for key, (s, e) in ddp.regions.items():
                self.pieces.append((s, e, key))
        n = sum(e - s for s, e, _ in self.pieces)
        pin = self.device.type == "cuda"
        self.master = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self.gbuf = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self.param_is_fp32 = ddp.param_data.dtype == torch.float32
        self.pbuf = (torch.empty(n, dtype=torch.int16, pin_memory=pin) if ddp.param_data.dtype == torch.bfloat16
                     else None)  # host bf16 (RNE) copy written by the kernel
        self.master_off = []
        o = 0
        with torch.no_grad():
            for s, e, _ in self.pieces:
                self.master[o:o + (e - s)].copy_(ddp.param_data[s:e].float())
                self.master_off.append(o)
                o += e - s
        self.found_inf = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.param_groups = [{"lr": lr, "weight_decay": weight_decay}]
        self._copy_stream = torch.cuda.Stream(self.device) if pin else None

    @torch.no_grad()
    def step(self, lr: Optional[float] = None):
        if lr is not None:
            self.lr = lr
        self.param_groups[0]["lr"] = self.lr
        _tp.params_changed()
        ddp = self.ddp
        ddp.wait_param_gather()
        g = ddp.grad_data
        self.found_inf.zero_()
        total = torch.zeros(1, dtype=torch.float64, device=self.device)   # order-insensitive sum of pieces
        for s, e, key in self.pieces:
            if e > s and (key[1] or self.scaler is not None):
                ss = self._sumsq(g[s:e])
                if key[1]:
                    total += ss
        for grp in self._norm_groups():
            dist.all_reduce(total, group=grp)
            dist.all_reduce(self.found_inf, op=dist.ReduceOp.MAX, group=grp)
        scale = float(self.scaler.scale.item()) if self.scaler is not None else 1.0
        norm = math.sqrt(float(total.item())) / scale
        inf = bool(self.found_inf.item())
        self.grad_norm = torch.tensor([norm], device=self.device)
        if self.scaler is not None:
            self.scaler.update(self.found_inf)
        if inf:
            return self.grad_norm
        coef = min(1.0, self.clip_grad / (norm + 1e-6)) if self.clip_grad > 0 else 1.0
        mul = coef / scale
        self.step_count += 1
        cuda = self.device.type == "cuda"
        # D2H all pieces on a side stream, event per piece, so host math on piece i overlaps copy i+1
        events = []
        cs = self._copy_stream
        if cuda:
            cs.wait_stream(torch.cuda.current_stream(self.device))
        for (s, e, _), mo in zip(self.pieces, self.master_off):
            if cuda:
                with torch.cuda.stream(cs):
                    self.gbuf[mo:mo + e - s].copy_(g[s:e], non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                events.append(ev)
            else:
                self.gbuf[mo:mo + e - s].copy_(g[s:e])
                events.append(None)
        for (s, e, key), mo, ev in zip(self.pieces, self.master_off, events):
            n = e - s
            if n <= 0:
                continue
            if ev is not None:
                ev.synchronize()
            wd = self.weight_decay if key[0] else 0.0
            out = 0 if self.pbuf is None else self.pbuf[mo:mo + n].data_ptr()
            self._rt.cpu_adam(self.master[mo:].data_ptr(), self.gbuf[mo:].data_ptr(), self.exp_avg[mo:].data_ptr(),
                              self.exp_avg_sq[mo:].data_ptr(), out, n, self.lr, self.beta1, self.beta2, self.eps,
                              wd, self.step_count, self.adamw, mul, self.threads)
            src = self.master[mo:mo + n] if self.pbuf is None else self.pbuf[mo:mo + n].view(torch.bfloat16)
            ddp.param_data[s:e].copy_(src.to(ddp.param_data.dtype) if src.dtype != ddp.param_data.dtype else src,
                                      non_blocking=cuda)
        if self.zero:
            ddp.all_gather_params()
        return self.grad_norm

    def state_dict(self):
        d = super().state_dict()
        d["offload"] = True
        return d

    def load_state_dict(self, d):
        self.step_count = int(d["step"])
        self.master.copy_(d["master"])
        self.exp_avg.copy_(d["exp_avg"])
        self.exp_avg_sq.copy_(d["exp_avg_sq"])
        self.lr = d.get("lr", self.lr)
        if self.scaler is not None and "scaler" in d:
            self.scaler.load_state_dict(d["scaler"])
        with torch.no_grad():
            for (s, e, _), mo in zip(self.pieces, self.master_off):
                self.ddp.param_data[s:e].copy_(self.master[mo:mo + (e - s)].to(self.ddp.param_data.dtype))
        if self.zero:
            self.ddp.all_gather_params()
