"""ZeRO stage 3: parameter partitioning with on-demand, prefetched all-gathers.

The reference's Alpaca job runs DeepSpeed ZeRO-3 with ``offload_param: cpu``
(/root/reference/4_training_alpaca_deepspeed/configs/default_offload_opt_param.json:23-41; the log
shows the partitioned init "num_elems = 0.16B", NB4:1580, and the offload, NB4:1629). This is the
MI355X-native equivalent, layered on the flat bucketed DDP buffers (parallel/distributed.py):

* every DP rank keeps only its shard of each parameter bucket (``store``: numel / dp elements, in
  HBM, or in pinned host memory with ``offload_param``); the full bucket exists only while a
  block that uses it runs;
* the model is cut into *blocks* — every child of an ``nn.ModuleList`` (a transformer layer) plus
  the root (embeddings, final norm, LM head); a block's forward / backward pre-hook gathers the
  buckets holding its parameters (one RCCL ``all_gather_into_tensor`` per bucket, the H2D copy
  of an offloaded shard first), its post-hook releases them; reference counts make nested and
  re-entrant use (activation recompute, the tied LM head inside the root) safe;
* the order in which buckets are first gathered is traced during the first forward and the
  first backward; later gathers prefetch the next buckets of that trace, up to
  ``prefetch_numel`` elements and at least the next block, so the gather of layer i + 1 runs
  beside the MFMA work of layer i (``stage3_prefetch_bucket_size``). The pinned-host H2D copy of
  an offloaded shard and the all-gather both run on the partitioner's side stream, and the compute
  stream waits for a bucket with a device-side event wait — the host never blocks on a gather;
* buckets whose parameters are all below ``persistence_threshold`` elements (biases, norms) stay
  gathered — re-gathered once after each optimizer step (``stage3_param_persistence_threshold``);
* gradients take the ZeRO-2 path of the DDP (bucket accumulation buffer -> reduce-scatter into
  the fp32 gradient shard), so gradient memory is ~ 1/dp as well.

Released parameters keep their Python objects with a 0-element placeholder as ``.data``;
autograd functions that saved the parameter itself (every linear / embedding / norm of the
model zoo does) see the re-gathered storage in backward.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .distributed import DistributedDataParallel, ShardedFlat, _is_dense


class ZeroParamPartitioner:
    def __init__(self, ddp: DistributedDataParallel, persistence_threshold: int = 0, prefetch_numel: int = 0,
                 offload: bool = False, max_live_numel: int = 0):
        if not (ddp.zero and ddp.zero_stage >= 3):
            raise ValueError("ZeroParamPartitioner needs DistributedDataParallel(use_distributed_optimizer=True, "
                             "zero_stage=3)")
        self.ddp = ddp
        self.dp = ddp.dp
        self.dev = ddp.grad_store.device
        self.dtype = ddp.param_dtype
        self.offload = bool(offload)
        self.prefetch_numel = int(prefetch_numel)
        # ``stage3_max_live_parameters``: a released bucket stays gathered while the gathered
        # (non-persistent) elements stay within this budget, so gradient-accumulation micro-batches
        # reuse the parameters gathered by the first one instead of re-fetching (and, offloaded,
        # re-copying from host) every layer twice per micro-batch; everything is dropped when the
        # optimizer is about to rewrite the shards (end_of_backward).
        self.max_live_numel = int(max_live_numel)
        self.live_numel = 0
        self.persistent = {b.index: max(ddp.param_index[id(p)][1] for p in b.params) <= persistence_threshold for b in ddp.buckets}
        total = sum(b.numel // self.dp for b in ddp.buckets)
        pin = self.offload and torch.cuda.is_available()
        self.store = torch.empty(total, dtype=self.dtype, device="cpu" if self.offload else self.dev,
                                 pin_memory=pin)
        self.full: Dict[int, torch.Tensor] = {}
        self.refs: Dict[int, int] = {b.index: 0 for b in ddp.buckets}
        self.inflight: Dict[int, tuple] = {}
        self.trace = {"fwd": [], "bwd": []}
        self._traced = {"fwd": False, "bwd": False}
        # H2D copies of offloaded shards and the parameter gathers run on a side stream, ordered by
        # events, so they overlap the compute of the previous block
        from ..comm.streams import comm_stream
        self.side = comm_stream(self.dev) if self.dev.type == "cuda" else None
        old = ddp.param_data
        with torch.no_grad():
            if ddp._zero_init:
                self._assemble_from_param_shards()
            else:
                for b in ddp.buckets:
                    s, e = ddp.shard_range(b)
                    self.store[b.shard_off:b.shard_off + (e - s)].copy_(old[s:e])
                    if self.persistent[b.index]:
                        self.full[b.index] = old[b.start:b.end].clone()
        ddp.param_data = ShardedFlat(ddp, self.store)
        ddp.zero3 = self
        for b in ddp.buckets:
            if self.persistent[b.index]:
                self._attach(b, self.full[b.index])
            else:
                self._detach(b)
        del old
        self._hooks = []
        self.blocks = self._find_blocks(ddp.module)
        for mod, bks in self.blocks:
            self._install(mod, bks, root=mod is ddp.module)
        self.block_numel = max((sum(ddp.buckets[i].numel for i in bks) for mod, bks in self.blocks
                                if mod is not ddp.module), default=0)

    def _assemble_from_param_shards(self):
        """Bucket shards from the per-parameter shards left by zero_init.Init: each parameter is
        all-gathered once (only ONE full parameter exists at a time), the part of it inside this
        rank's shard of its bucket is kept, and the per-parameter shard is dropped. Small
        (persistent) buckets keep their full copy, as in the resident path."""
        from . import zero_init as zi
        ddp = self.ddp
        for b in ddp.buckets:
            s, e = ddp.shard_range(b)
            fullbuf = torch.zeros(b.numel, dtype=self.dtype, device=self.dev) if self.persistent[b.index] else None
            for p in b.params:
                o, n = ddp.param_index[id(p)]
                full = (zi.gather_full(p, ddp.dp_group) if zi.is_partitioned(p) else p.data.reshape(-1)).to(self.dev, self.dtype)
                lo, hi = max(o, s), min(o + n, e)
                if lo < hi:
                    self.store[b.shard_off + (lo - s):b.shard_off + (hi - s)].copy_(full[lo - o:hi - o])
                if fullbuf is not None:
                    fullbuf[o - b.start:o - b.start + n].copy_(full)
                del full
                if zi.is_partitioned(p):
                    del p._zi_shard
                    del p._zi_shape
            if fullbuf is not None:
                self.full[b.index] = fullbuf

    # ------------------------------------------------------------------ layout
    def _find_blocks(self, root: nn.Module):
        """[(module, bucket indices)] — ModuleList children, then the root for everything else."""
        blocks: List[nn.Module] = []
        for m in root.modules():
            if isinstance(m, nn.ModuleList):
                blocks.extend(m.children())
        owned = set()
        out = []
        for blk in blocks:
            ids = {id(p) for p in blk.parameters() if id(p) in self.ddp.param_bucket}
            owned |= ids
            out.append((blk, sorted({self.ddp.param_bucket[i].index for i in ids})))
        rest = {id(p) for p in root.parameters() if id(p) in self.ddp.param_bucket} - owned
        out.append((root, sorted({self.ddp.param_bucket[i].index for i in rest})))
        return out

    def _install(self, mod: nn.Module, bks: List[int], root: bool):
        # The root's inputs are token ids: torch warns that its full backward pre-hook fires on
        # output gradients only — which is exactly when the root's buckets are needed.
        import warnings
        warnings.filterwarnings("ignore", message="Full backward hook is firing when gradients are computed with "
                                "respect to module outputs")
        acq_f = lambda *_: self.acquire(bks, "fwd")           # noqa: E731
        rel = lambda *_: self.release(bks)                     # noqa: E731
        acq_b = lambda *_: self.acquire(bks, "bwd")            # noqa: E731
        self._hooks.append(mod.register_forward_pre_hook(acq_f))
        self._hooks.append(mod.register_forward_hook(lambda *_: rel()))
        self._hooks.append(mod.register_full_backward_pre_hook(lambda *_: acq_b()))
        if not root:   # the root's inputs (token ids) carry no gradient: released at end_of_backward
            self._hooks.append(mod.register_full_backward_hook(lambda *_: rel()))

    def _views(self, b, buf):
        for p in b.params:
            o, n = self.ddp.param_index[id(p)]
            shape, stride = self.ddp.shapes[id(p)]
            flat = buf[o - b.start:o - b.start + n]
            yield p, (flat.view(shape) if _is_dense(shape, stride) else flat.as_strided(shape, stride))

    def _attach(self, b, buf):
        for p, v in self._views(b, buf):
            p.data = v

    def _detach(self, b):
        from .tensor_parallel import drop_cached_weight_t
        drop_cached_weight_t(b.params)      # the dgrad W^T cache must not outlive the gather
        ph = torch.empty(0, dtype=self.dtype, device=self.dev)
        for p in b.params:
            p.data = ph

    # ------------------------------------------------------------------ gathers
    def _gather_async(self, b):
        """Start materialising bucket b: (pinned host ->) device copy of this rank's shard and the
        all-gather, both on the partitioner's side stream after the compute stream's work so far
        (the optimizer's shard writes). Returns (ready event or work, full buffer)."""
        n = b.numel // self.dp
        shard = self.store[b.shard_off:b.shard_off + n]
        if self.side is None:
            buf = torch.empty(b.numel, dtype=self.dtype, device=self.dev)
            if self.dp == 1:
                buf.copy_(shard)
                return None, buf
            return dist.all_gather_into_tensor(buf, shard, group=self.ddp.dp_group, async_op=True), buf
        cur = torch.cuda.current_stream(self.dev)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            if self.offload:
                shard = shard.to(self.dev, non_blocking=True)     # H2D beside the compute stream
            buf = torch.empty(b.numel, dtype=self.dtype, device=self.dev)
            if self.dp == 1:
                buf.copy_(shard, non_blocking=True)
            else:
                dist.all_gather_into_tensor(buf, shard, group=self.ddp.dp_group)
            ev = torch.cuda.Event()
            ev.record(self.side)
        return ev, buf

    def _materialise(self, i):
        b = self.ddp.buckets[i]
        if i in self.full:
            return
        h, buf = self.inflight.pop(i) if i in self.inflight else self._gather_async(b)
        if isinstance(h, torch.cuda.Event):
            cur = torch.cuda.current_stream(self.dev)
            cur.wait_event(h)                 # a device-side wait: the host never blocks here
            buf.record_stream(cur)
        elif h is not None:
            h.wait()
        self.full[i] = buf
        self.live_numel += b.numel
        self._attach(b, buf)

    def _prefetch_after(self, i, phase):
        if self.prefetch_numel <= 0 or not self._traced.get(phase, False):
            return
        tr = self.trace[phase]
        try:
            k = tr.index(i)
        except ValueError:
            return
        # ``stage3_prefetch_bucket_size`` elements ahead, but never less than the next block's
        # buckets (DeepSpeed's "auto" 0.9 h^2 is a fraction of one transformer layer, which would
        # leave the next layer's gather exposed)
        budget = max(self.prefetch_numel, self.block_numel)
        for j in tr[k + 1:]:
            if budget <= 0:
                break
            if j in self.full or j in self.inflight or self.persistent[j]:
                continue
            self.inflight[j] = self._gather_async(self.ddp.buckets[j])
            budget -= self.ddp.buckets[j].numel

    @torch.no_grad()
    def acquire(self, bks, phase="fwd"):
        for i in bks:
            if self.persistent[i]:
                continue
            if phase in self.trace and not self._traced[phase] and i not in self.trace[phase]:
                self.trace[phase].append(i)
            self.refs[i] += 1
            self._materialise(i)
            self._prefetch_after(i, phase)

    def release(self, bks):
        for i in bks:
            if self.persistent[i]:
                continue
            self.refs[i] = max(self.refs[i] - 1, 0)
            if self.refs[i] == 0 and i in self.full and self.live_numel > self.max_live_numel:
                self._free(i)

    def _free(self, i):
        del self.full[i]
        self.live_numel -= self.ddp.buckets[i].numel
        self._detach(self.ddp.buckets[i])

    def end_of_forward_trace(self):
        self._traced["fwd"] = True

    def end_of_backward(self):
        """Called by the DDP when the gradient sync finished: drop what backward still holds and
        freeze the traces (the first iteration defines the prefetch order)."""
        for i, (h, buf) in list(self.inflight.items()):
            if isinstance(h, torch.cuda.Event):
                torch.cuda.current_stream(self.dev).wait_event(h)
                buf.record_stream(torch.cuda.current_stream(self.dev))
            elif h is not None:
                h.wait()
        self.inflight.clear()
        for i in list(self.full):
            if not self.persistent[i]:
                self.refs[i] = 0
                self._free(i)
        if self.trace["fwd"]:
            self._traced["fwd"] = True
        if self.trace["bwd"]:
            self._traced["bwd"] = True

    @torch.no_grad()
    def after_step(self):
        """The optimizer wrote new shards: refresh the persistent (always gathered) buckets."""
        for b in self.ddp.buckets:
            if self.persistent[b.index]:
                h, buf = self._gather_async(b)
                if isinstance(h, torch.cuda.Event):
                    torch.cuda.current_stream(self.dev).wait_event(h)
                    buf.record_stream(torch.cuda.current_stream(self.dev))
                elif h is not None:
                    h.wait()
                self.full[b.index].copy_(buf)

    @contextlib.contextmanager
    def gathered(self):
        """All parameters materialised (checkpoint save, state_dict, evaluation outside hooks)."""
        bks = [b.index for b in self.ddp.buckets]
        self.acquire(bks, "other")
        try:
            yield
        finally:
            self.release(bks)

    def param_memory_numel(self) -> Dict[str, int]:
        """Persistent parameter storage on this rank: the shard store (HBM or host) and the
        always-gathered small buckets."""
        pers = sum(self.ddp.buckets[i].numel for i, v in self.persistent.items() if v)
        return {"shard": self.store.numel(), "persistent": pers, "device": str(self.store.device)}

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def partition_parameters(ddp: DistributedDataParallel, persistence_threshold: int = 0, prefetch_numel: int = 0,
                         offload: bool = False, max_live_numel: int = 0) -> ZeroParamPartitioner:
    return ZeroParamPartitioner(ddp, persistence_threshold, prefetch_numel, offload, max_live_numel)
