"""Mixed-precision Adam/AdamW over the DDP flat buffers, with optional ZeRO sharding, grad
clipping and (dynamic) loss scaling — no host synchronisation inside ``step``.

Covers Megatron's ``Float16OptimizerWithFloat16Params`` + FusedAdam + clip + DynamicGradScaler
(flags `--optimizer adam --adam-beta1/2 --adam-eps --weight-decay
--clip-grad --loss-scale --initial-loss-scale --min-loss-scale --loss-scale-window --hysteresis`,
/root/reference/3_training_megatron-lm/megatron/arguments.py:700-714, :968-979), the distributed
optimizer (P7, `--use-distributed-optimizer`, :1059-1060) and DeepSpeed ZeRO-1/2 with FusedAdam
(P8, K10; /root/reference/4_training_alpaca_deepspeed/configs/default_offload_opt_param.json).

State layout: fp32 master weights, exp_avg, exp_avg_sq are flat buffers covering either the
whole DDP buffer (plain) or only this DP rank's shard of every bucket (ZeRO). Each step runs:

    sumsq (per region, HIP) -> [all-reduce over DP (ZeRO) / TP / PP] -> clip coefficient (device)
    -> fused Adam per region / bucket shard (reads grad_mul + found_inf from device memory,
       writes fp32 master AND the bf16 model copy) -> [ZeRO: all-gather bf16 params]

With ZeRO the gradient buffer is reduce-scattered bucket by bucket during backward (stage 2
style: only the owned shard of each bucket is needed after the collective).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..comm import health as _health
from ..comm import stats as _cs
from ..ops import _ext
from ..parallel import state as ps
from ..parallel.distributed import DistributedDataParallel
from ..parallel import tensor_parallel as _tp


class DynamicLossScaler:
    """Megatron's DynamicGradScaler: halve on overflow after ``hysteresis`` hits, grow x2
    every ``window`` clean steps; state lives on the device (no sync)."""

    def __init__(self, initial_scale=2.0 ** 32, min_scale=1.0, growth_factor=2.0, backoff_factor=0.5,
                 growth_interval=1000, hysteresis=2, device=None):
        self.scale = torch.tensor([float(initial_scale)], dtype=torch.float32, device=device)
        self.min_scale = float(min_scale)
        self.growth_factor, self.backoff_factor = growth_factor, backoff_factor
        self.growth_interval = int(growth_interval)
        self.hysteresis = int(hysteresis)
        self._hyst = torch.tensor([self.hysteresis], dtype=torch.int32, device=device)
        self._growth = torch.tensor([0], dtype=torch.int32, device=device)

    def update(self, found_inf):
        inf = found_inf.bool()
        self._hyst = torch.where(inf, self._hyst - 1, self._hyst)
        shrink = inf & (self._hyst <= 0)
        self.scale = torch.where(shrink, torch.clamp(self.scale * self.backoff_factor, min=self.min_scale), self.scale)
        self._growth = torch.where(inf, torch.zeros_like(self._growth), self._growth + 1)
        grow = self._growth >= self.growth_interval
        self.scale = torch.where(grow, self.scale * self.growth_factor, self.scale)
        self._growth = torch.where(grow, torch.zeros_like(self._growth), self._growth)
        self._hyst = torch.where(grow, torch.full_like(self._hyst, self.hysteresis), self._hyst)

    def state_dict(self):
        return {"scale": self.scale.cpu(), "hyst": self._hyst.cpu(), "growth": self._growth.cpu()}

    def load_state_dict(self, d):
        dev = self.scale.device
        self.scale = d["scale"].to(dev)
        self._hyst = d["hyst"].to(dev)
        self._growth = d["growth"].to(dev)


class ConstantLossScaler:
    def __init__(self, scale=1.0, device=None):
        self.scale = torch.tensor([float(scale)], dtype=torch.float32, device=device)

    def update(self, found_inf):
        pass

    def state_dict(self):
        return {"scale": self.scale.cpu()}

    def load_state_dict(self, d):
        self.scale = d["scale"].to(self.scale.device)


class MixedPrecisionAdam:
    def __init__(self, ddp: DistributedDataParallel, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, adamw: bool = True, clip_grad: float = 0.0,
                 loss_scaler=None, use_distributed_optimizer: Optional[bool] = None,
                 capturable: bool = False):
        """``capturable``: the step count, bias corrections and lr live on the device
        (``adam_capturable`` reads [lr, 1 - beta1^t, 1 - beta2^t] at run time), so the whole
        training step, optimizer included, can be captured in a HIP graph and replayed. Inside
        a capture the lr is not re-written (it would be baked in): change it between replays
        with ``set_lr``."""
        self.ddp = ddp
        self.lr = lr
        self.beta1, self.beta2 = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.adamw = adamw
        self.clip_grad = clip_grad
        self.zero = ddp.zero if use_distributed_optimizer is None else use_distributed_optimizer
        if self.zero and not ddp.zero:
            raise ValueError("ZeRO optimizer needs DistributedDataParallel(use_distributed_optimizer=True)")
        self.scaler = loss_scaler
        self.step_count = 0
        dev = ddp.grad_data.device   # ZeRO-3 + offload_param: the param shards live on the host
        self.device = dev
        # (start, end) pieces of the flat buffers this rank updates, with their region keys.
        self.pieces = []
        if self.zero:
            for b in ddp.buckets:
                s, e = ddp.shard_range(b)
                self.pieces.append((s, e, b.region))
        else:
            for key, (s, e) in ddp.regions.items():
                self.pieces.append((s, e, key))
        n = sum(e - s for s, e, _ in self.pieces)
        self.master = torch.empty(n, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.master_off = []
        o = 0
        with torch.no_grad():
            for s, e, _ in self.pieces:
                self.master[o:o + (e - s)].copy_(ddp.param_data[s:e].float())
                self.master_off.append(o)
                o += e - s
        self.param_is_fp32 = ddp.param_data.dtype == torch.float32
        self.found_inf = torch.zeros(1, dtype=torch.int32, device=dev)
        self.grad_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.capturable = bool(capturable) and dev.type == "cuda"
        if self.capturable:
            self._step_t = torch.zeros(1, dtype=torch.float32, device=dev)
            self._hyp = torch.tensor([lr, 1.0, 1.0], dtype=torch.float32, device=dev)
        self.param_groups = [{"lr": lr, "weight_decay": weight_decay}]
        # an xGMI engine that timed out NaN-filled gathered parameters: rewrite them from the
        # masters and re-gather over RCCL (comm/health.py)
        _health.on_fallback(self.repair_params)

    # ------------------------------------------------------------------ helpers
    def _norm_groups(self):
        st = ps.get_state()
        groups = []
        if self.zero and self.ddp.dp > 1:
            groups.append(self.ddp.dp_group)
        if st.mp_group is not None and (st.tp > 1 or st.pp > 1):
            groups.append(st.mp_group)
        return groups

    def _sumsq(self, x):
        if _ext.use_kernels(x):
            return _ext.ext().sumsq(x, self.found_inf)
        xf = x.float()
        if not torch.isfinite(xf).all():
            self.found_inf.fill_(1)
        # fp64 accumulation: the norm (hence the clip coefficient) does not depend on how the
        # gradient is split into pieces (ZeRO shards vs whole buckets) or on the reduction order
        return xf.double().square().sum().float().view(1)

    def _counted_sum(self, fn) -> torch.Tensor:
        """sum over this rank's counted pieces (regions whose params count toward the norm on this
        rank: TP-replicated params on TP rank 0, the shared embedding on the first stage) of
        fn(piece index, start, end), reduced over the grad-norm groups (ZeRO's DP group, TP x PP)."""
        tot = torch.zeros(1, dtype=torch.float64, device=self.device)
        for i, (s, e, key) in enumerate(self.pieces):
            if key[1] and e > s:
                tot += fn(i, s, e)
        for g in self._norm_groups():
            dist.all_reduce(tot, group=g)
        return tot

    def params_norm(self) -> float:
        """L2 norm of the model's parameters (``--log-params-norm``; Megatron's
        calc_params_l2_norm), from the fp32 masters; collective over the grad-norm groups."""
        def sq(i, s, e):
            o = self.master_off[i]
            return self.master[o:o + (e - s)].double().square().sum()
        return float(self._counted_sum(sq).sqrt().item())

    def num_zeros_in_grad(self) -> int:
        """Zero entries of the reduced gradients (``--log-num-zeros-in-grad``), over the same
        pieces and groups; call after the gradient sync."""
        g = self.ddp.grad_data
        return int(self._counted_sum(lambda i, s, e: (g[s:e] == 0).sum().double()).item())

    def zero_grad(self, set_to_none: bool = True):
        """torch.optim-style: a torch_compat DDP re-zeroes its flat gradient buffer on the next
        forward by itself; the explicit-step API zeroes it here."""
        if not getattr(self.ddp, "torch_compat", False):
            self.ddp.zero_grad_buffer()

    def set_lr(self, lr: float):
        """The learning rate of the next steps (outside a capture for a capturable optimizer)."""
        self.lr = float(lr)
        self.param_groups[0]["lr"] = self.lr
        if self.capturable:
            self._hyp[0:1].fill_(self.lr)

    @torch.no_grad()
    def step(self, lr: Optional[float] = None):
        """One optimizer step over the reduced gradients. Returns the device grad-norm tensor."""
        if lr is not None:
            self.lr = lr
        self.param_groups[0]["lr"] = self.lr
        if self.capturable:
            if not torch.cuda.is_current_stream_capturing():
                self._hyp[0:1].fill_(self.lr)
            self._step_t += 1                            # device step count: replays advance it
            self._hyp[1:2].copy_(1.0 - torch.pow(self.beta1, self._step_t))
            self._hyp[2:3].copy_(1.0 - torch.pow(self.beta2, self._step_t))
        _tp.params_changed()
        ddp = self.ddp
        if hasattr(ddp, "wait_param_gather"):
            ddp.wait_param_gather()          # (also the previous step's overlapped updates)
        g = ddp.grad_data
        self.found_inf.zero_()
        total = torch.zeros(1, dtype=torch.float64, device=self.device)   # order-insensitive sum of pieces
        for s, e, key in self.pieces:
            if key[1] and e > s:                        # counts toward the norm on this rank
                total += self._sumsq(g[s:e])
            elif e > s and self.scaler is not None:   # still check for inf/nan
                self._sumsq(g[s:e])
        for grp in self._norm_groups():
            with _cs.blocking("all_reduce", grp, 8):
                dist.all_reduce(total, group=grp)
                dist.all_reduce(self.found_inf, op=dist.ReduceOp.MAX, group=grp)
        inv_scale = 1.0
        scale_t = None
        if self.scaler is not None:
            scale_t = self.scaler.scale
        use_k = _ext.use_kernels(g)
        if use_k:
            mul, norm = _ext.ext().clip_coef(total.float(), float(self.clip_grad), 1.0)
            if scale_t is not None:
                mul = mul / scale_t
                norm = norm / scale_t
                if self.clip_grad > 0:
                    # clip coefficient must use the unscaled norm
                    coef = torch.clamp(self.clip_grad / (norm + 1e-6), max=1.0)
                    mul = coef / scale_t
        else:
            norm = torch.sqrt(total).float()
            if scale_t is not None:
                norm = norm / scale_t
            coef = torch.clamp(self.clip_grad / (norm + 1e-6), max=1.0) if self.clip_grad > 0 else torch.ones_like(norm)
            mul = coef / (scale_t if scale_t is not None else 1.0)
        self.grad_norm = norm
        self.step_count += 1
        t = self.step_count
        bc1 = 1 - self.beta1 ** t
        bc2 = 1 - self.beta2 ** t
        if (use_k and self.zero and getattr(ddp, "overlap_optimizer", False) and ddp.zero3 is None
                and not self.param_is_fp32 and len(self.pieces) == len(ddp.buckets) and not self.capturable
                and self._overlappable):
            self._step_overlapped(g, mul, t)
            if self.scaler is not None:
                self.scaler.update(self.found_inf)
            return self.grad_norm
        for (s, e, key), mo in zip(self.pieces, self.master_off):
            if e <= s:
                continue
            self._update_piece(g, s, e, key, mo, mul, use_k, t, bc1, bc2)
        if self.scaler is not None:
            self.scaler.update(self.found_inf)
        if self.zero:
            ddp.all_gather_params()
        return self.grad_norm

    _overlappable = True     # the per-bucket update may run on the overlapped side stream

    def _update_piece(self, g, s, e, key, mo, mul, use_k, t, bc1, bc2):
        """The fused (Adam / AdamW) update of one piece [s, e) of the flat buffers: fp32 master,
        moments, the model-dtype parameter copy; skipped (state untouched) on found_inf."""
        ddp = self.ddp
        n = e - s
        wd = self.weight_decay if key[0] else 0.0
        mst, m, v = self.master[mo:mo + n], self.exp_avg[mo:mo + n], self.exp_avg_sq[mo:mo + n]
        gr = g[s:e]
        if gr.dtype != torch.float32:
            gr = gr.float()
        if use_k:
            model_out = None if self.param_is_fp32 else ddp.param_data[s:e]
            host_out = None
            if model_out is not None and not model_out.is_cuda:   # offloaded ZeRO-3 param shard
                host_out, model_out = model_out, torch.empty(n, dtype=model_out.dtype, device=mst.device)
            if self.capturable:
                _ext.ext().adam_capturable(mst, gr, m, v, model_out, self._hyp, self.beta1, self.beta2,
                                           self.eps, wd, self.adamw, mul, self.found_inf)
            else:
                _ext.ext().adam(mst, gr, m, v, model_out, self.lr, self.beta1, self.beta2, self.eps, wd, t,
                                self.adamw, mul, self.found_inf)
            if host_out is not None:
                host_out.copy_(model_out)
            if self.param_is_fp32:
                ddp.param_data[s:e].copy_(mst)
        else:
            ok = (self.found_inf == 0).float()
            # an overflow step must leave every state untouched: inf * 0 would be NaN
            gg = torch.where(self.found_inf == 0, gr * mul, torch.zeros_like(gr))
            if not self.adamw and wd:
                gg = gg + wd * mst
            m.mul_(1 - (1 - self.beta1) * ok).add_(gg * ((1 - self.beta1) * ok))
            v.mul_(1 - (1 - self.beta2) * ok).add_(gg * gg * ((1 - self.beta2) * ok))
            denom = v.sqrt() / math.sqrt(bc2) + self.eps
            upd = (m / bc1) / denom
            if self.adamw and wd:
                upd = upd + wd * mst
            mst.sub_(self.lr * upd * ok)
            ddp.param_data[s:e].copy_(mst.to(ddp.param_data.dtype))

    def _step_overlapped(self, g, mul, t):
        """The fused AdamW of every bucket on a side stream, in the forward order DDP computed
        (``opt_bucket_order``), one event per bucket that the forward pre-hooks wait on; each
        bucket's gradients are zeroed right after its update (DDP.zero_grad_buffer skips them)."""
        ddp = self.ddp
        cur = torch.cuda.current_stream(self.device)
        if getattr(self, "_opt_stream", None) is None:
            self._opt_stream = torch.cuda.Stream(device=self.device)
        side = self._opt_stream
        side.wait_stream(cur)                  # the norm, the clip coefficient, found_inf
        delay = int(os.environ.get("SMDT_OPT_STREAM_DELAY", "0"))   # tests: widen the race window
        with torch.cuda.stream(side):
            for i in ddp.opt_bucket_order:
                if delay:
                    torch.cuda._sleep(delay)
                s, e, key = self.pieces[i]
                if e <= s:
                    continue
                mo, n = self.master_off[i], e - s
                wd = self.weight_decay if key[0] else 0.0
                gr = g[s:e]
                _ext.ext().adam(self.master[mo:mo + n], gr, self.exp_avg[mo:mo + n], self.exp_avg_sq[mo:mo + n],
                                ddp.param_data[s:e], self.lr, self.beta1, self.beta2, self.eps, wd, t, self.adamw,
                                mul, self.found_inf)
                gr.zero_()
                ev = torch.cuda.Event()
                ev.record(side)
                ddp._opt_events[i] = ev
        mul.record_stream(side)                # freed tensors must outlive the side-stream reads
        ddp._async_zeroed = True

    @torch.no_grad()
    def repair_params(self):
        """Model-dtype parameters <- fp32 masters for this rank's pieces, then (ZeRO) re-gather the
        full buffer: undoes NaN-filled parameter gathers after a collective timed out."""
        _tp.params_changed()
        ddp = self.ddp
        if hasattr(ddp, "wait_param_gather"):
            ddp.wait_param_gather()
        for (s, e, _), mo in zip(self.pieces, self.master_off):
            if e > s:
                ddp.param_data[s:e].copy_(self.master[mo:mo + (e - s)].to(ddp.param_data.dtype))
        if self.zero:
            ddp.all_gather_params()
            ddp.wait_param_gather()

    @torch.no_grad()
    def reload_model_params(self):
        """Refresh the fp32 masters from the model buffer (after loading weights only)."""
        _tp.params_changed()
        self.ddp.wait_param_gather()
        for (s, e, _), mo in zip(self.pieces, self.master_off):
            self.master[mo:mo + (e - s)].copy_(self.ddp.param_data[s:e].float())

    def get_loss_scale(self):
        return self.scaler.scale if self.scaler is not None else None

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self):
        self.ddp.wait_param_gather()         # an overlapped update may still be writing the state
        if self.capturable:                  # graph replays advance the device count only
            self.step_count = int(self._step_t.item())
        d = {"step": self.step_count, "master": self.master, "exp_avg": self.exp_avg,
             "exp_avg_sq": self.exp_avg_sq, "lr": self.lr, "zero": self.zero,
             "pieces": [(s, e) for s, e, _ in self.pieces]}
        if self.scaler is not None:
            d["scaler"] = self.scaler.state_dict()
        return d

    def load_state_dict(self, d):
        self.ddp.wait_param_gather()
        _tp.params_changed()
        self.step_count = int(d["step"])
        if self.capturable:
            self._step_t.fill_(self.step_count)
        self.master.copy_(d["master"])
        self.exp_avg.copy_(d["exp_avg"])
        if self.exp_avg_sq.numel():          # (SGD keeps no second moment)
            self.exp_avg_sq.copy_(d["exp_avg_sq"])
        self.lr = d.get("lr", self.lr)
        if self.scaler is not None and "scaler" in d:
            self.scaler.load_state_dict(d["scaler"])
        with torch.no_grad():
            for (s, e, _), mo in zip(self.pieces, self.master_off):
                self.ddp.param_data[s:e].copy_(self.master[mo:mo + (e - s)].to(self.ddp.param_data.dtype))
        if self.zero:
            self.ddp.all_gather_params()


class MixedPrecisionSGD(MixedPrecisionAdam):
    """``--optimizer sgd`` (Megatron's SGD path, /root/reference/3_training_megatron-lm/megatron/
    arguments.py ``--optimizer`` / ``--sgd-momentum``): momentum SGD, torch.optim.SGD semantics
    (buf = momentum * buf + g + wd * p; p -= lr * buf), over the same flat fp32 masters, gradient
    reduction, clipping, loss scaling and found-inf skip as the Adam path. The momentum buffer is
    ``exp_avg``; no second moment is kept. Elementwise torch ops (not a fused kernel): SGD is off
    the measured path."""

    _overlappable = False

    def __init__(self, ddp: DistributedDataParallel, lr: float = 1e-2, momentum: float = 0.9,
                 weight_decay: float = 0.0, clip_grad: float = 0.0, loss_scaler=None,
                 use_distributed_optimizer: Optional[bool] = None):
        super().__init__(ddp, lr=lr, weight_decay=weight_decay, adamw=False, clip_grad=clip_grad,
                         loss_scaler=loss_scaler, use_distributed_optimizer=use_distributed_optimizer)
        self.momentum = float(momentum)
        self.exp_avg_sq = torch.empty(0, dtype=torch.float32, device=self.device)

    def _update_piece(self, g, s, e, key, mo, mul, use_k, t, bc1, bc2):
        ddp = self.ddp
        n = e - s
        wd = self.weight_decay if key[0] else 0.0
        mst, buf = self.master[mo:mo + n], self.exp_avg[mo:mo + n]
        gr = g[s:e].float()
        ok = self.found_inf == 0
        gg = torch.where(ok, gr * mul, torch.zeros_like(gr))
        if wd:
            gg = gg + wd * mst
        buf.copy_(torch.where(ok, buf * self.momentum + gg, buf))
        mst.sub_(self.lr * buf * ok.float())
        out = ddp.param_data[s:e]
        out.copy_(mst.to(out.dtype) if out.device == mst.device else mst.to(out.device, out.dtype))
