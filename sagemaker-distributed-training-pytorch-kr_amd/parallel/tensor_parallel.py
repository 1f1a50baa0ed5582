"""Megatron-style tensor and sequence parallelism over RCCL.

Equivalent of ``megatron.core.tensor_parallel`` as exercised by the reference recipe (SURVEY P4,
P6, K7, K13, U4: Column/RowParallelLinear, VocabParallelEmbedding, broadcast_data, the async
TP all-reduce `megatron/arguments.py:837-842`, sequence parallelism `:848-849` and gradient
accumulation fusion `:850-854` in /root/reference/3_training_megatron-lm).

Design notes (MI355X-first):
  * Weight gradients are accumulated straight into the fp32 ``param.main_grad`` view of the
    contiguous DDP buffer (K7), after which the layer tells the DDP reducer the parameter is
    ready, so the bucket's RCCL all-reduce / reduce-scatter launches while backward continues.
  * The input-gradient collective (TP all-reduce, or the SP reduce-scatter) is issued
    asynchronously and overlapped with the weight-gradient GEMM.
  * Weights are initialised from a TP-invariant generator (full tensor, then this rank's shard)
    so a TP=k model starts bit-identical to the TP=1 model: this is what the parallel-equivalence
    tests rely on.
"""
from __future__ import annotations

import contextlib
import hashlib
import math
import os
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..comm import loopback as _lb
from ..comm import relay as _relay
from ..comm import stats as _cs
from ..ops import _ext
from ..ops import functional as SF
from . import state as ps

# --------------------------------------------------------------------------------------------
# collectives helpers


def _tp_size():
    return ps.get_state().tp


def _tp_group():
    return ps.get_state().tp_group


def _nbytes(t):
    return t.numel() * t.element_size()


def _all_reduce(x, group, async_op=False):
    if dist.get_world_size(group) == 1:
        return None
    if not async_op:
        eng = ps.xgmi_engine(group)  # xGMI IPC all-reduce (comm/xgmi.py) when enabled for the group
        if eng is not None and eng.use["all_reduce"] and eng.fits(x):
            with _cs.blocking("all_reduce", group, _nbytes(x), "xgmi"):
                done = eng.all_reduce(x)
            if done:
                return None
        with _cs.blocking("all_reduce", group, _nbytes(x)):
            return dist.all_reduce(x, group=group)
    h = dist.all_reduce(x, group=group, async_op=True)
    _cs.collective("all_reduce", group, _nbytes(x), work=h)
    return h


def _gather_dim0(x, group):
    ws = dist.get_world_size(group)
    if ws == 1:
        return x
    out = torch.empty((x.shape[0] * ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    with _cs.blocking("all_gather", group, _nbytes(out)):
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
    return out


def _reduce_scatter_dim0(x, group, async_op=False):
    ws = dist.get_world_size(group)
    if ws == 1:
        return x, None
    assert x.shape[0] % ws == 0, "sequence length must divide the TP size"
    out = torch.empty((x.shape[0] // ws,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    if not async_op:
        with _cs.blocking("reduce_scatter", group, _nbytes(x)):
            dist.reduce_scatter_tensor(out, x.contiguous(), group=group)
        return out, None
    h = dist.reduce_scatter_tensor(out, x.contiguous(), group=group, async_op=True)
    _cs.collective("reduce_scatter", group, _nbytes(x), work=h)
    return out, h


# CUs held by in-flight exchanges (id(work) -> workgroups): the relay engine's kernel (and its
# paced single-GPU stand-in) keeps 2 x world x sub workgroups resident for the whole transfer, one
# per CU (a GEMM workgroup fills a CU's register file, so neither can share a CU). A persistent
# GEMM launched beside it with one workgroup per CU (gemm_tn) would leave that many of its
# workgroups waiting for the transfer to end — or, launched first, keep the transfer from starting
# until the GEMM's tail: measured with the paced stand-in as ~every exchange fully exposed
# (profiles/r6_standin/). Chunk GEMMs issued while an exchange is in flight size their grid to
# the CUs left over (``gemm_tn_blocks``). SMDT_EXCHANGE_CU_RESERVE=0 turns this off.
_CU_HELD = {}
_CU_RESERVE_ON = os.environ.get("SMDT_EXCHANGE_CU_RESERVE", "1") == "1"
_NUM_CUS = []


def _hold_cus(works, blocks):
    if _CU_RESERVE_ON and blocks > 0:
        for w in works:
            _CU_HELD[id(w)] = int(blocks)


def gemm_tn_blocks() -> int:
    """max_blocks for a persistent gemm_tn launch now: 0 (every CU) unless exchanges in flight hold
    CUs, then the CUs they leave."""
    if not _CU_HELD:
        return 0
    if not _NUM_CUS:
        _NUM_CUS.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    # max, not sum: the exchanges in flight run one after another on their engine's stream
    return max(_NUM_CUS[0] - max(_CU_HELD.values()), _NUM_CUS[0] // 2)


def _wait_works(works, group):
    """Wait (on the current stream) for in-flight works of ``group``'s collectives."""
    for w in works:
        _CU_HELD.pop(id(w), None)
    if not _cs._ON:
        for w in works:
            w.wait()
        return
    with _cs.waiting(_cs.axis_of(group)):
        for w in works:
            w.wait()


def _split_dim(x, dim, group):
    ws = dist.get_world_size(group)
    if ws == 1:
        return x
    r = dist.get_rank(group)
    return x.chunk(ws, dim=dim)[r].contiguous()


def _gather_dim(x, dim, group):
    ws = dist.get_world_size(group)
    if ws == 1:
        return x
    if dim == 0:
        return _gather_dim0(x, group)
    parts = [torch.empty_like(x) for _ in range(ws)]
    dist.all_gather(parts, x.contiguous(), group=group)
    return torch.cat(parts, dim=dim)


class _CopyToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        _all_reduce(g, _tp_group())
        return g


class _ReduceFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        _all_reduce(x, _tp_group())
        return x

    @staticmethod
    def backward(ctx, g):
        return g


class _ScatterToTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _split_dim(x, -1, _tp_group())

    @staticmethod
    def backward(ctx, g):
        return _gather_dim(g, -1, _tp_group())


class _GatherFromTP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _gather_dim(x, -1, _tp_group())

    @staticmethod
    def backward(ctx, g):
        return _split_dim(g, -1, _tp_group())


class _ScatterToSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _split_dim(x, 0, _tp_group())

    @staticmethod
    def backward(ctx, g):
        return _gather_dim0(g, _tp_group())


class _GatherFromSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, tp_output_grad):
        ctx.tp_output_grad = tp_output_grad
        return _gather_dim0(x, _tp_group())

    @staticmethod
    def backward(ctx, g):
        if ctx.tp_output_grad:
            return _reduce_scatter_dim0(g, _tp_group())[0], None
        return _split_dim(g, 0, _tp_group()), None


class _ReduceScatterToSP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return _reduce_scatter_dim0(x, _tp_group())[0]

    @staticmethod
    def backward(ctx, g):
        return _gather_dim0(g, _tp_group())


def copy_to_tensor_model_parallel_region(x):
    return _CopyToTP.apply(x) if _tp_size() > 1 else x


def reduce_from_tensor_model_parallel_region(x):
    return _ReduceFromTP.apply(x) if _tp_size() > 1 else x


def scatter_to_tensor_model_parallel_region(x):
    return _ScatterToTP.apply(x) if _tp_size() > 1 else x


def gather_from_tensor_model_parallel_region(x):
    return _GatherFromTP.apply(x) if _tp_size() > 1 else x


def scatter_to_sequence_parallel_region(x):
    return _ScatterToSP.apply(x) if _tp_size() > 1 else x


def gather_from_sequence_parallel_region(x, tensor_parallel_output_grad=True):
    return _GatherFromSP.apply(x, tensor_parallel_output_grad) if _tp_size() > 1 else x


def reduce_scatter_to_sequence_parallel_region(x):
    return _ReduceScatterToSP.apply(x) if _tp_size() > 1 else x


# --------------------------------------------------------------------------------------------
# Linear with async grad communication + fused fp32 wgrad accumulation (K7)


_FUSED_WGRAD = os.environ.get("SMDT_FUSED_WGRAD", "1") == "1"
# Which fused fp32-accumulate wgrad GEMM runs: "mfma" (hand-written gfx950 kernel,
# csrc/kernels/wgrad_gemm.hip), "blaslt" (hipBLASLt beta = 1) or "auto" (time both once per shape
# on scratch buffers and keep the faster). The MFMA kernel measured faster than hipBLASLt on every
# GPT-2 345M shape (BENCHMARKS.md), so it is the default.
_WGRAD_IMPL = os.environ.get("SMDT_WGRAD_IMPL", "mfma")
_WGRAD_CHOICE = {}


def _time_us(fn, reps=3):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def _wgrad_impl(C, mg, g2, t2):
    if _WGRAD_IMPL != "auto" or g2.dtype not in (torch.bfloat16, torch.float16):
        return _WGRAD_IMPL if g2.dtype in (torch.bfloat16, torch.float16) else "blaslt"
    key = (g2.shape[0], g2.shape[1], t2.shape[1], g2.device.index)
    impl = _WGRAD_CHOICE.get(key)
    if impl is None:
        scratch = torch.zeros_like(mg)
        impl = "blaslt"
        if C.wgrad_mfma(scratch, g2, t2, 0):
            tm = _time_us(lambda: C.wgrad_mfma(scratch, g2, t2, 0))
            tb = _time_us(lambda: C.wgrad_accumulate(scratch, g2, t2))
            impl = "mfma" if tm < tb else "blaslt"
        _WGRAD_CHOICE[key] = impl
    return impl


class DeferredWgrad:
    """Deferred, grouped weight-gradient GEMMs.

    Backward produces one wgrad GEMM per linear layer; on their own the small ones (the 1024 x
    1024 attention projection, the QKV GEMM) cannot fill 256 CUs without split-K, and split-K
    pays fp32 atomics (~1.3 TB/s chip-wide). Instead ``_wgrad`` queues (main_grad, dY, X) and
    the queue is flushed as ONE grouped launch of the gfx950 MFMA kernel
    (csrc/kernels/wgrad_gemm.hip, ``smdt_wgrad_grouped``): every tile runs over the full token
    range, no atomics, deterministic. The queue holds dY / X alive until the flush (a few hundred
    MB per layer at GPT-2 345M scale: trivial next to 288 GB of HBM), flushes once it holds
    ``flush_tiles`` output tiles (several layers, so gradient buckets still become ready while
    backward runs and DDP overlaps their RCCL reduction), and is drained by DDP's
    ``start/finish_grad_sync`` before any gradient is read. A weight is reported ready to DDP
    only when its GEMM has been issued. Tensors are version-checked at flush time: an in-place
    write into a queued dY or X raises instead of producing a wrong gradient.
    """

    def __init__(self):
        self.enabled = os.environ.get("SMDT_DEFER_WGRAD", "1") == "1"
        self.flush_tiles = int(os.environ.get("SMDT_DEFER_WGRAD_TILES", "1024"))
        # Gradient-accumulation window (set by the ZeRO engine, train/zero.py): while ``hold`` is
        # on, nothing flushes on size and DDP's sync re-enable does not drain the queue, so the
        # GEMMs of ALL micro-batches of a window meet in the queue. A weight queued again is
        # MERGED (its dY / X segments are concatenated along the token dim at flush time): one
        # GEMM over the window's tokens and ONE read-modify-write of the fp32 main_grad instead of
        # one per micro-batch (LLaMA-7B: 54 GB of main_grad traffic per pass). Held dY / X are
        # capped at SMDT_WGRAD_HOLD_GB, by default a quarter of the device memory free at the
        # first push (then the queue flushes as usual).
        self.hold = False
        self.hold_bytes_cap = None      # set at the first push (_hold_cap)
        self.allow_cpu = False          # tests: exercise the queue logic with a torch fallback
        # Split backward (the zero-bubble pipeline schedules, train/schedules.py): while ``defer``
        # is on, nothing flushes on size and the opportunistic flushes inside backward (beside an
        # in-flight TP collective) are skipped, so a stage's whole backward pass is B (the input
        # gradient chain) and its weight-gradient GEMMs (W) run only when the schedule flushes,
        # after the input gradient was sent to the previous stage.
        self.defer = False
        # Merged items of a held window: concatenate the segments (one GEMM over all tokens, one
        # main_grad read-modify-write: the SFT engine's small micro-batches) or issue one grouped
        # launch per segment round (large pipeline micro-batches: no concatenation copy).
        self.concat_segments = True
        # the sub-batch interleave (models/transformer._forward_subbatch) pushes every weight twice
        # per pass (once per batch half): merge the second push instead of flushing, the segments
        # issued as rounds (no concatenation copy)
        self.merge_repeats = False
        self.ready_after_join = []      # filler-stream items waiting for their readiness report
        self.stats = {"flushes": 0, "items": 0, "max_segments": 0, "stores": 0}
        self.items = []
        self.by_key = {}
        self.tiles = 0
        self.held_bytes = 0

    @property
    def targets(self):
        return set(self.by_key)

    def eligible(self, mg, g2, t2):
        if not self.enabled or mg.dtype != torch.float32 or not mg.is_contiguous():
            return False
        if g2.dim() != 2 or t2.dim() != 2:
            return False
        M, N, K = g2.shape[0], g2.shape[1], t2.shape[1]
        if M % 32 or N % 8 or K % 8 or mg.numel() != N * K:
            return False
        if g2.is_cuda:
            return (_FUSED_WGRAD and g2.dtype in (torch.bfloat16, torch.float16) and t2.dtype == g2.dtype
                    and _ext.use_kernels(g2))
        return self.allow_cpu

    def _hold_cap(self, dev) -> int:
        env = os.environ.get("SMDT_WGRAD_HOLD_GB")
        if env is not None:
            return int(float(env) * 2 ** 30)
        if dev.type == "cuda":
            return int(0.25 * torch.cuda.mem_get_info(dev)[0])
        return 64 * 2 ** 30

    def push(self, weight, mg, g2, t2, bias=None, fresh=False):
        """Queue mg += g2^T t2; ``bias`` (a bias Parameter with an fp32 main_grad, or None): its
        gradient, the column sums of g2, comes out of the same grouped launch. ``fresh``: mg holds
        no data yet (a lazily zeroed ZeRO-2 gradient buffer) — the first GEMM into it stores
        instead of adding."""
        if self.hold_bytes_cap is None:
            self.hold_bytes_cap = self._hold_cap(g2.device)
        key = mg.data_ptr()
        g2, t2 = g2.contiguous(), t2.contiguous()
        seg = (g2, t2, g2._version, t2._version)
        nbytes = g2.numel() * g2.element_size() + t2.numel() * t2.element_size()
        it = self.by_key.get(key)
        if it is not None and (it[3] or self.hold or self.merge_repeats):
            # the same main_grad again inside an accumulation window: merge (the sum over the
            # concatenated token range is the same accumulation; one readiness report)
            it[2].append(seg)
            it[4] = it[4] or not self.hold
        else:
            if it is not None:          # same main_grad twice outside a window: keep order
                self.flush()
            # [weight, main_grad, segments, held (created inside a window), has its segment of
            # the synchronising pass, bias parameter or None, main_grad unwritten (store)]
            it = [weight, mg, [seg], self.hold, not self.hold, bias, bool(fresh)]
            self.items.append(it)
            self.by_key[key] = it
            self.tiles += -(-g2.shape[1] // 256) * -(-t2.shape[1] // 256)
        self.held_bytes += nbytes
        if self.held_bytes > self.hold_bytes_cap:
            self.flush()
        elif not self.hold and not self.defer:
            # size trigger on what a flush would issue now (the complete items): held items still
            # waiting for this pass's gradient neither count nor flush
            ready = [x for x in self.items if x[4]]
            tiles = sum(-(-x[2][0][0].shape[1] // 256) * -(-x[2][0][1].shape[1] // 256) for x in ready)
            if tiles >= self.flush_tiles or len(ready) >= 32:
                self.flush(complete_only=True)

    def flush_opportunistic(self):
        """A flush placed beside an in-flight collective to overlap it; skipped while ``defer``."""
        if not self.defer:
            self.flush()

    @torch.no_grad()
    def flush(self, complete_only: bool = False):
        """Issue the queued GEMMs (one grouped launch) and report readiness. ``complete_only`` (the
        size-triggered flush of a synchronising pass): items of a held window whose weight has
        not yet received this pass's gradient stay queued to merge with it. A held item flushed
        without that gradient (a forced flush) accumulates but reports no readiness: the pass's
        own item for the weight does."""
        if not self.items:
            return
        if complete_only:
            items = [it for it in self.items if it[4]]
            keep = [it for it in self.items if not it[4]]
        else:
            items, keep = self.items, []
        if not items:
            return
        self.items = keep
        self.by_key = {it[1].data_ptr(): it for it in keep}
        self.tiles = sum(-(-it[2][0][0].shape[1] // 256) * -(-it[2][0][1].shape[1] // 256) for it in keep)
        self.held_bytes = sum(sg[0].numel() * sg[0].element_size() + sg[1].numel() * sg[1].element_size()
                              for it in keep for sg in it[2])
        work = []
        for weight, mg, segs, _held, complete, bias, fresh in items:
            for g2, t2, vg, vt in segs:
                if g2._version != vg or t2._version != vt:
                    raise RuntimeError("deferred wgrad: a queued dY / X tensor was modified in place before the "
                                       "flush; disable with SMDT_DEFER_WGRAD=0 and report the op that did it")
            if len(segs) == 1:
                work.append((weight, mg, [(segs[0][0], segs[0][1])], complete, bias, fresh))
            elif self.concat_segments and _held:
                work.append((weight, mg, [(torch.cat([sg[0] for sg in segs]), torch.cat([sg[1] for sg in segs]))],
                             complete, bias, fresh))
            else:
                work.append((weight, mg, [(sg[0], sg[1]) for sg in segs], complete, bias, fresh))
        self.stats["flushes"] += 1
        self.stats["items"] += len(work)
        self.stats["max_segments"] = max(self.stats["max_segments"], max(len(w[2]) for w in work))
        # round i issues the i-th segment of every item: one grouped launch per round, so two
        # segments of one main_grad never run in the same launch (no write race, no atomics)
        for i in range(max(len(w[2]) for w in work)):
            # round 0 of an unwritten main_grad stores (overwrite), later rounds add
            rnd = [(mg, sg[i], b, fr and i == 0) for _, mg, sg, _, b, fr in work if len(sg) > i]
            self.stats["stores"] += sum(1 for r in rnd if r[3])
            cuda = [(mg, g2, t2, b, ow) for mg, (g2, t2), b, ow in rnd if g2.is_cuda]
            done = False
            if cuda:
                bts = [b.main_grad if b is not None else _NO_BIAS.get(g2.device) for _, g2, _, b, _ in cuda]
                done = _ext.ext().wgrad_grouped([c[0] for c in cuda], [c[1] for c in cuda], [c[2] for c in cuda], bts,
                                                [c[4] for c in cuda])
            for mg, (g2, t2), b, ow in rnd:
                if not (g2.is_cuda and done):
                    prod = g2.t().matmul(t2).view_as(mg)
                    if ow:
                        mg.copy_(prod)
                    else:
                        mg.add_(prod)
                    if b is not None:
                        b.main_grad.add_(g2.float().sum(0))
        for weight, _, _, complete, b, _ in work:
            if not complete:
                continue
            for p in (weight, b):
                cb = getattr(p, "_smdt_grad_ready", None) if p is not None else None
                if cb is not None:
                    cb(p)


    @torch.no_grad()
    def fill_one(self, cus: int = 0) -> bool:
        """Exchange-wait filler (``fill``): issue the oldest queued, complete and not held item —
        ONE weight's gradient GEMM — as its own grouped launch sized for ``cus`` CUs (the ones an
        in-flight TP exchange leaves; its tail split into pieces that fill them), and report its
        readiness. Returns False when there was nothing to issue."""
        pick = next((it for it in self.items if it[4] and not it[3]), None)
        if pick is None:
            return False
        self.items = [it for it in self.items if it is not pick]
        self.by_key.pop(pick[1].data_ptr(), None)
        weight, mg, segs, _held, _complete, bias, fresh = pick
        self.tiles -= -(-segs[0][0].shape[1] // 256) * -(-segs[0][1].shape[1] // 256)
        self.held_bytes -= sum(sg[0].numel() * sg[0].element_size() + sg[1].numel() * sg[1].element_size()
                               for sg in segs)
        for g2, t2, vg, vt in segs:
            if g2._version != vg or t2._version != vt:
                raise RuntimeError("deferred wgrad: a queued dY / X tensor was modified in place before the "
                                   "flush; disable with SMDT_DEFER_WGRAD=0 and report the op that did it")
        bt = bias.main_grad if bias is not None else _NO_BIAS.get(mg.device)
        for i, (g2, t2, _, _) in enumerate(segs):      # segments in order: round 0 may store
            ow = bool(fresh) and i == 0
            if g2.is_cuda and _FILL_IMPL == "blaslt":
                # hipBLASLt beta = 1 into main_grad (its own non-persistent tiling shares the CUs
                # with the transfer without a tail split) + the bias column sums
                C = _ext.ext()
                if ow:
                    mg.zero_()
                if not C.wgrad_accumulate(mg, g2, t2):
                    raise RuntimeError("deferred wgrad filler: hipBLASLt wgrad refused")
                if bias is not None:
                    C.bias_grad(g2, bias.main_grad, True)
                continue
            if g2.is_cuda:
                if not _ext.ext().wgrad_grouped([mg], [g2], [t2], [bt], [ow], int(cus)):
                    raise RuntimeError("deferred wgrad filler: grouped launch refused")
                continue
            prod = g2.t().matmul(t2).view_as(mg)       # CPU (tests: allow_cpu)
            if ow:
                mg.copy_(prod)
            else:
                mg.add_(prod)
            if bias is not None:
                bias.main_grad.add_(g2.float().sum(0))
        self.stats["fills"] = self.stats.get("fills", 0) + 1
        for p in (weight, bias):
            cb = getattr(p, "_smdt_grad_ready", None) if p is not None else None
            if cb is not None:
                cb(p)
        return True

    @torch.no_grad()
    def fill_many(self, budget_us: float, cus: int = 0, stream=None) -> int:
        """Exchange-wait filler, grouped form: the oldest queued, complete, not held, single-segment
        CUDA items up to ~``budget_us`` of estimated GEMM time (at least one) as ONE grouped launch
        sized for ``cus`` CUs. ``stream``: issue it there (the filler stream: it then never delays
        the next exchange, which waits only for the compute stream) — the caller joins that stream
        and ``fire_ready`` reports the items' readiness afterwards. Returns the items issued."""
        picks, spent = [], 0.0
        for it in self.items:
            if not (it[4] and not it[3] and len(it[2]) == 1 and it[1].is_cuda):
                continue
            if picks and spent + _item_us(it, cus) > budget_us:
                break
            picks.append(it)
            spent += _item_us(it, cus)
            if spent >= budget_us:
                break
        if not picks:
            return 0
        ids = {id(it) for it in picks}
        self.items = [it for it in self.items if id(it) not in ids]
        for it in picks:
            self.by_key.pop(it[1].data_ptr(), None)
            g2, t2, vg, vt = it[2][0]
            if g2._version != vg or t2._version != vt:
                raise RuntimeError("deferred wgrad: a queued dY / X tensor was modified in place before the "
                                   "flush; disable with SMDT_DEFER_WGRAD=0 and report the op that did it")
            self.tiles -= -(-g2.shape[1] // 256) * -(-t2.shape[1] // 256)
            self.held_bytes -= g2.numel() * g2.element_size() + t2.numel() * t2.element_size()
        mgs = [it[1] for it in picks]
        g2s = [it[2][0][0] for it in picks]
        t2s = [it[2][0][1] for it in picks]
        bts = [it[5].main_grad if it[5] is not None else _NO_BIAS.get(it[1].device) for it in picks]
        ows = [bool(it[6]) for it in picks]
        if stream is not None:
            for t in g2s + t2s:
                t.record_stream(stream)      # the queue drops them before the filler stream ran
        if not _ext.ext().wgrad_grouped(mgs, g2s, t2s, bts, ows, int(cus)):
            raise RuntimeError("deferred wgrad filler: grouped launch refused")
        self.stats["fills"] = self.stats.get("fills", 0) + len(picks)
        ready = [p for it in picks for p in (it[0], it[5]) if p is not None]
        if stream is None:
            self._fire(ready)
        else:
            self.ready_after_join.extend(ready)
        return len(picks)

    def fire_ready(self):
        """Readiness of the items issued on the filler stream (after the caller joined it)."""
        ready, self.ready_after_join = self.ready_after_join, []
        self._fire(ready)

    @staticmethod
    def _fire(params):
        for p in params:
            cb = getattr(p, "_smdt_grad_ready", None)
            if cb is not None:
                cb(p)

    def flush_unheld(self):
        """Issue every queued item that is not held for a later synchronising pass."""
        if not any(not it[3] for it in self.items):
            return
        held = [it for it in self.items if it[3]]
        if not held:
            self.flush()
            return
        self.items = [it for it in self.items if not it[3]]
        self.flush()
        self.items = held + self.items
        self.by_key = {it[1].data_ptr(): it for it in self.items}
        self.tiles = sum(-(-it[2][0][0].shape[1] // 256) * -(-it[2][0][1].shape[1] // 256) for it in self.items)
        self.held_bytes = sum(sg[0].numel() * sg[0].element_size() + sg[1].numel() * sg[1].element_size()
                              for it in self.items for sg in it[2])


DEFERRED_WGRAD = DeferredWgrad()
# Exchange-wait fillers (SMDT_W_FILL=1, split-backward pipeline schedules): the W GEMMs of the last
# backward pass stay queued into the next forward, whose TP-exchange waits each issue one of them
# (``fill_exchange_wait``) beside the in-flight transfer, on the CUs the transfer leaves; the rest
# is flushed when that forward ends (train/schedules.py). VERDICT r5 item 1, "split-K W fillers".
W_FILL = os.environ.get("SMDT_W_FILL", "0") == "1"
# W GEMM time offered to one exchange wait (us): ~ the relay's 131 us per 33.6 MB chunk less the
# chunk GEMM beside it; fillers are priced at _FILL_PFLOPS over the CUs the exchange leaves
_FILL_STREAM_ON = os.environ.get("SMDT_W_FILL_STREAM", "1") == "1"
# on the filler stream a filler may outlast its exchange without delaying the next one: 250 us
# measured best there (profiles/r6_fill3/: 110 / 250 / 500 us), 110 us on the compute stream
_FILL_US = float(os.environ.get("SMDT_W_FILL_US", "250" if _FILL_STREAM_ON else "110"))
_FILL_PFLOPS = 1.0
_FILL_IMPL = os.environ.get("SMDT_W_FILL_IMPL", "grouped")     # "grouped" (MFMA, split tail) / "blaslt"
_FILL = {"on": False}


def _item_us(it, cus):
    g2, t2 = it[2][0][0], it[2][0][1]
    fl = 2.0 * g2.shape[0] * g2.shape[1] * t2.shape[1] * len(it[2])
    return fl / (_FILL_PFLOPS * 1e9 * max(cus or 256, 1) / 256.0)


# SMDT_W_FILL_STREAM (default 1, above): the fillers go to a stream of their own (joined at the end
# of each pass), so a filler that outlasts its exchange no longer holds up the next exchange's start
_FILL_STREAMS = {}


def _fill_stream(dev):
    s = _FILL_STREAMS.get(dev)
    if s is None:
        s = _FILL_STREAMS[dev] = torch.cuda.Stream(dev)
    return s


def fill_exchange_wait():
    """Before a ring exchange's wait (forward or backward): issue queued W GEMMs beside the
    transfer, oldest first, up to ~_FILL_US of estimated GEMM time."""
    if not (_FILL["on"] and DEFERRED_WGRAD.items):
        return
    cus = gemm_tn_blocks()
    it0 = next((x for x in DEFERRED_WGRAD.items if x[4] and not x[3]), None)
    if it0 is not None and it0[1].is_cuda and len(it0[2]) == 1:
        if _FILL_STREAM_ON:
            dev = it0[1].device
            fs = _fill_stream(dev)
            fs.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(fs):
                DEFERRED_WGRAD.fill_many(_FILL_US, cus, stream=fs)
        else:
            DEFERRED_WGRAD.fill_many(_FILL_US, cus)
        return
    spent = 0.0
    while spent < _FILL_US:
        it = next((x for x in DEFERRED_WGRAD.items if x[4] and not x[3]), None)
        if it is None:
            return
        spent += _item_us(it, cus)
        DEFERRED_WGRAD.fill_one(cus)


def join_fill_stream():
    """The compute stream waits for the filler stream; then the filled items report readiness."""
    if _FILL_STREAMS:
        for dev, fs in _FILL_STREAMS.items():
            torch.cuda.current_stream(dev).wait_stream(fs)
    if DEFERRED_WGRAD.ready_after_join:
        DEFERRED_WGRAD.fire_ready()


class forward_fill:
    """Context for one pass (``flush_end``: a forward) of a split-backward schedule under
    SMDT_W_FILL: exchange waits take W fillers; after a forward, whatever is left unheld is
    flushed (a backward leaves its own W queued for the next forward)."""

    def __init__(self, flush_end: bool = True):
        self.flush_end = flush_end

    def __enter__(self):
        self.prev = _FILL["on"]
        _FILL["on"] = W_FILL
        return self

    def __exit__(self, *exc):
        _FILL["on"] = self.prev
        if W_FILL:
            join_fill_stream()
            if self.flush_end:
                DEFERRED_WGRAD.flush_unheld()
        return False


class _NoBias(dict):
    """Per-device empty fp32 tensor: 'no bias target' in a grouped wgrad launch's bias list."""

    def get(self, dev):
        t = super().get(dev)
        if t is None:
            t = self[dev] = torch.empty(0, dtype=torch.float32, device=dev)
        return t


_NO_BIAS = _NoBias()


def flush_deferred_wgrad():
    DEFERRED_WGRAD.flush()


def reset_wgrad_window():
    """Leave hold mode and issue whatever is queued (end of a training loop, or one that stopped
    inside an accumulation window)."""
    DEFERRED_WGRAD.hold = False
    DEFERRED_WGRAD.flush()


def accumulation_window_ok(ddps, default: bool = True) -> bool:
    """Whether gradient accumulation over these DDP wrappers may hold + merge the micro-batches'
    deferred wgrad GEMMs (DeferredWgrad.hold): the no_sync micro-batches must report no readiness
    (stage 0 / 1, or stage 2 writing its single DP rank's gradient store in place), no ZeRO-3
    partitioner, no pipeline. SMDT_WGRAD_MERGE_ACCUM=1 / 0 forces it on / off; otherwise
    ``default`` decides. It pays for small micro-batches, where every micro-batch's wgrad is a
    short K-loop plus a full fp32 main_grad read-modify-write (LLaMA-7B at ~500 tokens: +12 %,
    profiles/r3_merge/), and costs for large ones, where the segment concatenation outweighs the
    saved main_grad traffic (GPT-2 small at 12,288 tokens per micro-batch: 75.5 vs 63.2 ms,
    profiles/r3_l4l/) — so the SFT engine defaults it on and the Megatron schedule off."""
    env = os.environ.get("SMDT_WGRAD_MERGE_ACCUM")
    if (env == "0" or (env is None and not default)) or not DEFERRED_WGRAD.enabled:
        return False
    if ps.get_state().pp != 1:
        return False
    for d in ddps:
        if getattr(d, "zero3", None) is not None:
            return False
        if getattr(d, "zero_stage", 0) >= 2 and not getattr(d, "_direct", False):
            return False
    return True


def accumulate_wgrad(mg, g2, t2):
    """mg (fp32 [N, K]) += g2^T t2 now: the MFMA wgrad kernel or hipBLASLt beta = 1, whichever the
    per-shape timing picked (no deferral, no readiness callback)."""
    done = False
    if (_FUSED_WGRAD and mg.dtype == torch.float32 and g2.dtype in (torch.bfloat16, torch.float16)
            and g2.is_cuda and mg.is_contiguous()):
        C = _ext.ext()
        g2, t2 = g2.contiguous(), t2.contiguous()
        if _wgrad_impl(C, mg, g2, t2) == "mfma":
            done = C.wgrad_mfma(mg, g2, t2, 0)
        if not done:
            done = C.wgrad_accumulate(mg, g2, t2)
    if not done:
        mg.add_(g2.t().matmul(t2).view_as(mg))


def _wgrad(weight, g2, t2):
    """dW = g2^T t2. With a DDP ``main_grad`` the product is accumulated straight into the fp32
    buffer (K7 gradient-accumulation fusion): queued for the grouped MFMA launch
    (``DeferredWgrad``), or ONE GEMM now (the MFMA kernel or hipBLASLt with beta = 1) instead of a
    bf16 GEMM + a separate fp32 add pass. Returns the gradient to hand back to autograd (None
    when it goes to ``main_grad``)."""
    raw = getattr(weight, "_smdt_mg_raw", None)     # lazily zeroed ZeRO-2 buffer (distributed.py)
    mg = raw() if raw is not None else getattr(weight, "main_grad", None)
    if mg is None:
        return g2.t().matmul(t2)
    if DEFERRED_WGRAD.eligible(mg, g2, t2):
        DEFERRED_WGRAD.push(weight, mg, g2, t2, fresh=raw is not None and weight._smdt_mg_claim())
        return None
    if raw is not None:
        mg = weight.main_grad                          # zeroes the slice if it is still unwritten
    accumulate_wgrad(mg, g2, t2)
    cb = getattr(weight, "_smdt_grad_ready", None)
    if cb is not None:
        cb(weight)
    return None


# The bias gradient of a column-parallel linear (the column sums of dY) comes out of the grouped
# wgrad launch that reads dY anyway (csrc/kernels/wgrad_gemm.hip ``bias``) instead of a separate
# pass over dY; SMDT_WGRAD_BIAS=0 keeps the separate column-sum kernel.
_WGRAD_BIAS = os.environ.get("SMDT_WGRAD_BIAS", "1") == "1"


def _wgrad_and_bias(weight, bias_p, g2, t2):
    """(dW, db) for autograd: dW = g2^T t2 and db = sum_rows g2, each None when it went straight
    into the parameter's fp32 main_grad (queued, or by a kernel now)."""
    if bias_p is not None and _WGRAD_BIAS and g2.is_cuda:
        raw = getattr(weight, "_smdt_mg_raw", None)
        mg = raw() if raw is not None else getattr(weight, "main_grad", None)
        tgt = SF.grad_accumulate_target(bias_p)
        if mg is not None and tgt is not None and tgt.numel() == g2.shape[-1] and DEFERRED_WGRAD.eligible(mg, g2, t2):
            DEFERRED_WGRAD.push(weight, mg, g2, t2, bias=bias_p,
                                fresh=raw is not None and weight._smdt_mg_claim())
            return None, None
    dw = _wgrad(weight, g2, t2)
    return dw, (_bias_grad(bias_p, g2) if bias_p is not None else None)


# dgrad layout: dX = dY W with W [out, in] row-major is hipBLASLt's "NN" GEMM on this ROCm build,
# 14-24 % slower than the "TN" GEMM the forward runs in (F.linear, W^T read K-contiguous). A
# contiguous W^T made by the LDS tile-transpose kernel (ops: transpose2d, ~25 us per GPT-2 345M
# layer) turns every dgrad into F.linear(dY, W^T): 42.5 -> 37.4 ms of dgrad per step at 64 x 1024
# tokens (benchmarks/bench_dgrad.py, profiles/r2_dgrad_tn/). The copy is made per backward call
# (no cache to invalidate when the optimizer or a checkpoint load rewrites the weight).
_DGRAD_TN = os.environ.get("SMDT_DGRAD_TN", "1") == "1"


# W^T is kept from the first backward that needs it until the parameters next change, so gradient
# accumulation (NB4: 8 micro-batches per step) and pipeline micro-batches transpose each weight
# once per optimizer step instead of once per micro-batch (LLaMA-7B: 27 GB of transpose traffic
# per micro-batch). Entries are keyed on the weight's storage and version counter, and the whole
# cache is dropped by ``params_changed()``, which every optimizer step / parameter repair / master
# reload calls before it writes parameters (those writes go through raw kernels that do not bump
# version counters). SMDT_DGRAD_WT_CACHE=0 transposes per call.
_WT_CACHE_ON = os.environ.get("SMDT_DGRAD_WT_CACHE", "1") == "1"
_WT_CACHE: dict = {}


def params_changed():
    """Invalidate every cached W^T (call before any out-of-autograd parameter write)."""
    _WT_CACHE.clear()


def drop_cached_weight_t(params):
    """Forget the W^T of these parameters (ZeRO-3 frees a gathered bucket: its transposes must go
    with it, or the cache would end up holding a full bf16 copy of the model on every rank)."""
    for p in params:
        _WT_CACHE.pop(id(p), None)


def mm_rows(g, w):
    """g @ w (NN), row-split like ``linear_rows`` (the dgrad form when no W^T is made)."""
    M = g.numel() // g.shape[-1]
    bl = _row_blocks(M) if g.is_cuda else None
    if bl is None:
        return g.matmul(w)
    g2 = g.reshape(M, g.shape[-1])
    out = g.new_empty(tuple(g.shape[:-1]) + (w.shape[1],))
    o2 = out.view(M, w.shape[1])
    for a, b in bl:
        torch.mm(g2[a:b], w, out=o2[a:b])
    return out


def _dgrad_weight_t(weight):
    """W^T [in, out] contiguous for the TN dgrad, or None to use dY @ W directly. (A per-shape
    timed NN-vs-TN pick for few-token backward passes measured neutral on the SFT recipe,
    profiles/r4_sft_dgrad_tn/: TN stays.)"""
    if (_DGRAD_TN and weight.is_cuda and weight.dim() == 2 and weight.is_contiguous()
            and weight.dtype in (torch.bfloat16, torch.float16)
            and weight.shape[0] % 8 == 0 and weight.shape[1] % 8 == 0
            and _ext.use_kernels(weight)):   # raises on a GPU box without the extension
        if not _WT_CACHE_ON:
            return _ext.ext().transpose2d(weight)
        key = (weight.data_ptr(), weight._version, tuple(weight.shape), weight.dtype)
        hit = _WT_CACHE.get(id(weight))
        if hit is not None and hit[0] == key:
            return hit[1]
        wt = _ext.ext().transpose2d(weight)
        _WT_CACHE[id(weight)] = (key, wt)
        return wt
    return None


# Row-split GEMMs. hipBLASLt's heuristic picks poor kernels for token counts just above a multiple
# of 4096 (the SFT recipe's packed windows: M ~ 4.3 k varies every step, so no per-shape tuning
# applies): LLaMA-7B layer GEMMs at M = 4300 run at 845 TF/s whole and 1207 TF/s as 4096 rows +
# the remainder (4608: 927 -> 1206, 8600: 1087 -> 1309; at 5000 / 6100 the whole GEMM is as fast
# or faster; benchmarks/bench_sft_gemm_split.py, profiles/r4_sft_gemm_split/). So a GEMM whose
# M exceeds a multiple of SMDT_GEMM_ROW_SPLIT (4096; 0 = off) by at most a sixth of it is issued
# as two row blocks into one output.
_ROW_SPLIT = int(os.environ.get("SMDT_GEMM_ROW_SPLIT", "4096"))


def _row_blocks(M: int):
    q = _ROW_SPLIT
    if q <= 0 or M <= q:
        return None
    r = M % q
    if r == 0 or r > q // 6:
        return None
    return ((0, M - r), (M - r, M))


# Hand-written MFMA GEMM (csrc/kernels/gemm_tn.hip: persistent 256 x 256 tiles, LDS-DMA stage
# ring, trickled epilogue stores) for out = x W^T where it beats hipBLASLt. SMDT_GEMM_TN: "0" off,
# "1" every supported shape, a comma list of "N:K" pairs (e.g. "4096:1024,1024:4096") for those
# shapes only. The fused fc1 + bias-GeLU op (``linear_bias_gelu``) is governed separately by
# SMDT_FUSED_BIAS_GELU.
_GEMM_TN = os.environ.get("SMDT_GEMM_TN", "0")


def _gemm_tn_shapes():
    if _GEMM_TN in ("0", "", "1"):
        return None
    out = set()
    for item in _GEMM_TN.split(","):
        n, k = item.split(":")
        out.add((int(n), int(k)))
    return out


_GEMM_TN_SHAPES = _gemm_tn_shapes()


def _gemm_tn_ok(x2, w, bias):
    if _GEMM_TN == "0" or not x2.is_cuda or w.dim() != 2:
        return False
    if bias is not None and (bias.dtype != x2.dtype or not bias.is_contiguous()):
        return False
    if _GEMM_TN_SHAPES is not None and (w.shape[0], w.shape[1]) not in _GEMM_TN_SHAPES:
        return False
    return _ext.ext().gemm_tn_supported(x2, w)


def linear_rows(x, w, bias=None):
    """F.linear(x, w, bias), split into row blocks when ``_row_blocks`` says the whole GEMM would
    take a slow hipBLASLt kernel (CUDA only; identical results: each row's dot products are the
    same); the hand-written gemm_tn where SMDT_GEMM_TN selects it."""
    if x.is_cuda and x.dim() >= 2:
        M = x.numel() // x.shape[-1]
        if x.is_contiguous():
            x2 = x.view(M, x.shape[-1])
            if _gemm_tn_ok(x2, w, bias):
                y = _ext.ext().gemm_tn(x2, w, 1 if bias is not None else 0, bias)[0]
                return y.view(tuple(x.shape[:-1]) + (w.shape[0],))
        bl = _row_blocks(M)
        if bl is not None:
            x2 = x.reshape(M, x.shape[-1])
            out = x.new_empty(tuple(x.shape[:-1]) + (w.shape[0],))
            o2 = out.view(M, w.shape[0])
            for a, b in bl:
                if bias is not None:
                    torch.addmm(bias, x2[a:b], w.t(), out=o2[a:b])
                else:
                    torch.mm(x2[a:b], w.t(), out=o2[a:b])
            return out
    return F.linear(x, w, bias)


def dgrad(g, weight, wt=None):
    """dX = g @ weight (g [..., out], weight [out, in]); ``wt`` = weight^T from _dgrad_weight_t."""
    if wt is None:
        return mm_rows(g, weight)
    return linear_rows(g, wt)


def dgrad_into(dst, g, weight, wt=None):
    """dst[...] = g @ weight written in place."""
    if wt is None:
        torch.matmul(g, weight, out=dst)
    else:
        _mm_into(dst, g, wt)


class LinearWithGradAccumulationAndAsyncCommunication(torch.autograd.Function):
    """y = x W^T (+ b) with Megatron's backward schedule:

    dgrad GEMM -> launch (async) TP all-reduce or SP reduce-scatter of dgrad -> wgrad GEMM into
    fp32 main_grad -> wait. With ``sequence_parallel`` the input is all-gathered along the
    sequence dim in forward (and re-gathered in backward, saving memory).
    """

    @staticmethod
    def forward(ctx, x, weight, bias, sequence_parallel, async_grad_allreduce, add_bias=True):
        ctx.sp = sequence_parallel
        ctx.async_ar = async_grad_allreduce
        ctx.has_bias = bias is not None
        ctx.bias_p = bias
        ctx.save_for_backward(x, weight)
        total = _gather_dim0(x, _tp_group()) if sequence_parallel else x
        # add_bias False: the caller adds the bias later (skip_bias_add) and this function only
        # produces its gradient (the column sums of dY) beside the weight gradient
        return linear_rows(total, weight, bias if add_bias else None)

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        gi_out, dw, db = _linear_backward(ctx, g, x, weight)
        return gi_out, dw, db, None, None, None


def _linear_backward(ctx, g, x, weight):
    """dgrad -> async TP all-reduce / SP reduce-scatter of it -> wgrad (+ bias grad) into the fp32
    main_grad -> wait: the backward of ``LinearWithGradAccumulationAndAsyncCommunication`` (ctx
    carries sp, async_ar, has_bias, bias_p)."""
    group = _tp_group()
    tp = dist.get_world_size(group) if group is not None else 1
    total = _gather_dim0(x, group) if (ctx.sp and tp > 1) else x
    g = g.contiguous()
    gi = dgrad(g, weight, _dgrad_weight_t(weight))
    handle = None
    if ctx.sp and tp > 1:
        gi_out, handle = _reduce_scatter_dim0(gi, group, async_op=True)
    else:
        gi_out = gi
        if ctx.async_ar and tp > 1:
            handle = _all_reduce(gi_out, group, async_op=True)
    g2 = g.reshape(-1, g.shape[-1])
    t2 = total.reshape(-1, total.shape[-1])
    dw, db = _wgrad_and_bias(weight, ctx.bias_p if ctx.has_bias else None, g2, t2)
    if handle is not None:
        # the collective is in flight: run the queued weight-gradient GEMMs beside it
        DEFERRED_WGRAD.flush_opportunistic()
        _wait_works([handle], group)
    return gi_out, dw, db


# fc1 + bias + GeLU(tanh) as ONE GEMM launch (gemm_tn.hip EPI_BIAS_GELU): the epilogue writes the
# pre-activation (kept for the backward) and the activation; the separate bias_act_fwd pass over
# the [tokens, 4h] tensor is gone (Megatron's bias_gelu_fusion,
# /root/reference/3_training_megatron-lm/megatron/arguments.py:819-821); at TP = 1 the backward's
# GeLU half goes into the fc2 dgrad's epilogue as well (FusedGeLUMLP). On by default: the GPT-2
# 345M step measured 160.45 / 161.06 / 160.64 ms against 160.67 / 160.68 / 161.01 ms unfused (one
# box, interleaved; profiles/r5_gemm_tn/) — the fused ops are 1.02x / 1.05x the library GEMM +
# elementwise pass, the hand-written GEMM itself 0.85-0.92x hipBLASLt. SMDT_FUSED_BIAS_GELU=0 off.
_FUSED_BIAS_GELU = os.environ.get("SMDT_FUSED_BIAS_GELU", "1") == "1"


class LinearBiasGeLU(torch.autograd.Function):
    """act = gelu_tanh(x W^T + b) for a column-parallel fc1 without sequence parallelism. Backward:
    d(pre) = bias_act_bwd(d(act), pre) (the bias gradient comes from the wgrad launch, as for
    ``ColumnParallelLinear(bias_grad_from_output=True)``), then the linear's own backward."""

    @staticmethod
    def forward(ctx, x, weight, bias, async_grad_allreduce):
        ctx.sp = False
        ctx.async_ar = async_grad_allreduce
        ctx.has_bias = True
        ctx.bias_p = bias
        x2 = x.reshape(-1, x.shape[-1])
        pre, act = _ext.ext().gemm_tn(x2, weight, 2, bias)
        ctx.save_for_backward(x, weight, pre)
        shape = tuple(x.shape[:-1]) + (weight.shape[0],)
        return act.view(shape)

    @staticmethod
    def backward(ctx, dact):
        x, weight, pre = ctx.saved_tensors
        d2 = dact.reshape(-1, dact.shape[-1]).contiguous()
        dpre = _ext.ext().bias_act_bwd(d2, pre, ctx.bias_p.detach(), 0, False, None)[0]
        gi, dw, db = _linear_backward(ctx, dpre.view(tuple(x.shape[:-1]) + (weight.shape[0],)), x, weight)
        return gi, dw, db, None


class FusedGeLUMLP(torch.autograd.Function):
    """fc2(gelu_tanh(fc1(x) + b1)) at TP = 1 with both GeLU halves inside the GEMMs (gemm_tn.hip):
    forward fc1 + bias + GeLU in one launch (EPI_BIAS_GELU), backward fc2's dgrad with the GeLU
    backward in its epilogue (EPI_DGELU: d(pre) = (dY W2) * gelu'(pre + b1), the [tokens, 4h]
    d(activation) is never written). Saves x, pre and act — what the unfused path saves. fc2's bias
    is added by the caller (skip_bias_add), as in ``ParallelMLP``. Same math as Megatron's
    ParallelMLP with bias_gelu_fusion (/root/reference/3_training_megatron-lm/megatron/
    arguments.py:819-821)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2):
        C = _ext.ext()
        x2 = x.reshape(-1, x.shape[-1])
        pre, act = C.gemm_tn(x2, w1, 2, b1)
        y = linear_rows(act, w2)
        ctx.save_for_backward(x, w1, w2, pre, act)
        ctx.b1 = b1
        return y.view(tuple(x.shape[:-1]) + (w2.shape[0],))

    @staticmethod
    def backward(ctx, dy):
        x, w1, w2, pre, act = ctx.saved_tensors
        C = _ext.ext()
        b1 = ctx.b1
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        w2t = _dgrad_weight_t(w2)
        if w2t is not None and C.gemm_tn_supported(dy2, w2t):
            dz = C.gemm_tn(dy2, w2t, 3, b1.detach(), None, None, 0, 0, pre)[0]
        else:
            dz = C.bias_act_bwd(dgrad(dy2, w2, w2t).contiguous(), pre, b1.detach(), 0, False, None)[0]
        dw2, _ = _wgrad_and_bias(w2, None, dy2, act)
        x2 = x.reshape(-1, x.shape[-1])
        dx = dgrad(dz, w1, _dgrad_weight_t(w1))
        dw1, db1 = _wgrad_and_bias(w1, b1, dz, x2)
        return dx.view(x.shape), dw1, db1, dw2


def fused_gelu_mlp_ok(x, mlp) -> bool:
    """``FusedGeLUMLP`` applies: the fc1 + bias-GeLU conditions, TP = 1, fc2 without sequence
    parallelism and with its bias left to the caller."""
    return (_tp_size() == 1 and linear_bias_gelu_ok(x, mlp.fc1) and mlp.fc2.skip_bias_add
            and not mlp.fc2.sequence_parallel and mlp.fc2.weight.dtype == x.dtype)


class SPFusedGeLUMLP(torch.autograd.Function):
    """The sequence-parallel MLP of a TP > 1 rank with both GeLU halves inside the ring-chunk GEMMs
    (the TP form of ``FusedGeLUMLP``; BASELINE config 3's tp2 + SP layers):

      forward   fc1: ring all-gather of the SP chunks of x, each chunk's GEMM with the bias-GeLU
                epilogue (gemm_tn EPI_BIAS_GELU) writing its rows of the pre-activation and the
                activation; fc2: per-chunk GEMMs fused with the ring reduce-scatter (as
                ``_RowSPLinear``);
      backward  fc2: ring all-gather of dY, each chunk's dgrad with the GeLU backward in its
                epilogue (EPI_DGELU) writing d(pre) directly — the [tokens, 4h / tp] d(activation)
                and the separate bias_act_bwd pass are gone; fc1: dgrad chunks fused with the ring
                reduce-scatter, the fc1 weight and bias gradients (one grouped-wgrad pass over
                d(pre)) drained while the last chunk is in flight (as ``_ColumnSPLinear``).

    The collectives, their order and the saved tensors (gathered x, pre, act) are those of the
    unfused column / row SP linears, so a TP group whose ranks disagree on the gate could not
    deadlock on the exchanges either (the gate depends on shapes and dtypes only). Megatron's
    ParallelMLP with bias_gelu_fusion + sequence_parallel (/root/reference/3_training_megatron-lm/
    megatron/arguments.py:819-821, 848-849)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2):
        C = _ext.ext()
        group = _tp_group()
        x = x.contiguous()
        n = x.shape[0]
        ws = dist.get_world_size(group)
        lead = (n * ws,) + tuple(x.shape[1:-1])
        f = w1.shape[0]
        pre = x.new_empty(lead + (f,))
        act = x.new_empty(lead + (f,))

        def fc1_chunk(lo, ch):
            m = ch.shape[0]
            C.gemm_tn(ch.reshape(-1, ch.shape[-1]), w1, 2, b1, pre[lo:lo + m].view(-1, f),
                      act[lo:lo + m].view(-1, f), gemm_tn_blocks())
        total = ag_ring(x, group, fc1_chunk)
        y = rs_ring(lambda lo, m, o: _linear_into(act[lo:lo + m], w2, o), group, lead + (w2.shape[0],), act)
        ctx.save_for_backward(total, w1, w2, pre, act)
        ctx.b1 = b1
        ctx.bulk = _SPLIT["on"]     # a sub-batch half: bulk rings in backward
        ctx.defer_add = _bwd_add_to_norm(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        total, w1, w2, pre, act = ctx.saved_tensors
        C = _ext.ext()
        group = _tp_group()
        b1 = ctx.b1
        dy = dy.contiguous()
        f = w1.shape[0]
        dz = pre.new_empty(pre.shape)
        d2 = dz.view(-1, f)
        w2t = _dgrad_weight_t(w2)
        bd = b1.detach()

        def fc2_dgrad_chunk(lo, ch):
            m = ch.shape[0]
            C.gemm_tn(ch.reshape(-1, ch.shape[-1]), w2t, 3, bd, dz[lo:lo + m].view(-1, f), None,
                      gemm_tn_blocks(), 0, pre[lo:lo + m].view(-1, f))
        gfull = ag_ring(dy, group, fc2_dgrad_chunk, before_last_wait=_flush_wgrad, bulk=ctx.bulk)
        dw2 = _wgrad(w2, gfull.reshape(-1, gfull.shape[-1]), act.reshape(-1, f))
        res = {}

        def wgrad():
            res["dw"], res["db"] = _wgrad_and_bias(w1, b1, d2, total.reshape(-1, total.shape[-1]))
            _flush_wgrad()
        w1t = _dgrad_weight_t(w1)
        dx = rs_ring(lambda lo, m, o: _dgrad_rows(dz[lo:lo + m], w1, w1t, o), group,
                     dz.shape[:-1] + (w1.shape[1],), dz, wgrad, bulk=ctx.bulk, defer_add=ctx.defer_add)
        if "dw" not in res:
            wgrad()
        return dx, res["dw"], res["db"], dw2


def sp_fused_gelu_mlp_ok(x, mlp) -> bool:
    """``SPFusedGeLUMLP`` applies: TP > 1 with the ring collective-matmul sequence-parallel linears,
    fc1 with a bias and fc2 with its bias left to the caller, 16-bit CUDA operands, and every chunk
    GEMM on a gemm_tn shape (SP-chunk rows and the local 4h a multiple of 256, h of 128).
    Depends on shapes / dtypes / flags only, so every rank of the TP group decides alike."""
    fc1, fc2 = mlp.fc1, mlp.fc2
    if not (_FUSED_BIAS_GELU and _TP_OVERLAP and _tp_size() > 1 and x.is_cuda and fc1.sequence_parallel
            and fc2.sequence_parallel and fc1.bias is not None and fc1.bias_grad_from_output
            and fc2.skip_bias_add and not fc1.gather_output and x.dtype in (torch.bfloat16, torch.float16)
            and fc1.weight.dtype == x.dtype and fc2.weight.dtype == x.dtype and fc1.bias.dtype == x.dtype
            and _ext.use_kernels(x)):
        return False
    if _direct(_tp_group()) is not None:   # the direct TP4 / TP8 engine hands over row pieces
        return False
    rows = x.numel() // x.shape[-1]
    f, h = fc1.weight.shape
    return (rows % 256 == 0 and f % 256 == 0 and h % 128 == 0 and fc2.weight.shape == (h, f)
            and _fills_chip(rows, f) and bool(_ext.ext().gemm_tn_supported(x.reshape(rows, h), fc1.weight)))


def _fills_chip(rows: int, n: int) -> bool:
    """A chunk GEMM of rows x n has at least one 256 x 256 output tile per CU: gemm_tn's
    persistent grid is one workgroup per tile up to the CU count, so fewer tiles leave CUs idle
    (GPT-3 6.7B tp4 + SP: 2048-row chunks x 4096 = 128 tiles -> the stage rank 426 ms with the
    fused MLP vs 394 ms on hipBLASLt, profiles/r6_ab/)."""
    if not _NUM_CUS:
        _NUM_CUS.append(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count)
    return (rows // 256) * (n // 256) >= _NUM_CUS[0]


def linear_bias_gelu_ok(x, layer) -> bool:
    """The fused fc1 + bias + GeLU path applies: CUDA, 16-bit, no sequence parallelism, a bias, and
    a shape gemm_tn supports."""
    if not (_FUSED_BIAS_GELU and x.is_cuda and layer.bias is not None and not layer.sequence_parallel
            and x.dtype in (torch.bfloat16, torch.float16) and layer.weight.dtype == x.dtype
            and layer.bias.dtype == x.dtype and x.is_contiguous() and not layer.gather_output
            and _ext.use_kernels(x)):
        return False
    x2 = x.view(-1, x.shape[-1])
    return _fills_chip(x2.shape[0], layer.weight.shape[0]) and bool(_ext.ext().gemm_tn_supported(x2, layer.weight))


def linear_bias_gelu(x, layer):
    """gelu_tanh(fc1(x) + b) through ``LinearBiasGeLU`` (call only when ``linear_bias_gelu_ok``)."""
    if not layer.async_ar:
        x = copy_to_tensor_model_parallel_region(x)
    return LinearBiasGeLU.apply(x, layer.weight, layer.bias, layer.async_ar)


class LMHeadCrossEntropy(torch.autograd.Function):
    """Per-token CE of ``h W^T`` for an unsplit vocab (TP = 1), the LM head and the loss as ONE op.

    The forward runs the logits GEMM, then ``ce_fused`` reads each logits row once and overwrites
    it with softmax - onehot (cross_entropy.hip). The backward applies the per-row dloss on the
    [tokens, hidden] side instead of the [tokens, vocab] side: dX = diag(dloss) (D W) and
    dW = D^T (diag(dloss) X), so no pass over the logits remains in the backward. Against the
    separate ce_stats / ce_bwd kernels this removes one full read of the logits per step. Same
    math as Megatron's LM head + vocab-parallel CE at TP = 1 (SURVEY K12 / K13;
    /root/reference/3_training_megatron-lm/pretrain_gpt.py:51-57).
    """

    @staticmethod
    def forward(ctx, h, weight, target, ignore_index, vvalid):
        logits = linear_rows(h, weight)
        loss = _ext_mod().ce_fused(logits.view(-1, logits.shape[-1]), target.contiguous().view(-1),
                                   int(ignore_index), int(vvalid))
        ctx.save_for_backward(h, weight, logits)
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, dloss):
        h, weight, d = ctx.saved_tensors
        dl = dloss.contiguous().view(-1, 1).float()
        gi = dgrad(d, weight, _dgrad_weight_t(weight))
        gi.view(-1, gi.shape[-1]).mul_(dl)
        hs = torch.mul(h.reshape(-1, h.shape[-1]), dl).to(h.dtype)
        dw = _wgrad(weight, d.view(-1, d.shape[-1]), hs)
        return gi, dw, None, None, None


def ce_local_pass(logits2d, target, vstart: int, vvalid: int):
    """One pass over this rank's vocab slice of the logits: overwrite them with e = exp(x - m_local)
    (0 on padding columns >= vvalid) and return the row statistics [3, rows] fp32 = (m_local,
    sum e, target logit if the target is in [vstart, vstart + vvalid) else 0). HIP kernel
    (cross_entropy.hip ce_fused_kernel<LOCAL>) on the GPU, the same math in PyTorch on the CPU."""
    if logits2d.is_cuda:
        return _ext_mod().ce_fused_local(logits2d, target, int(vstart), int(vvalid))
    V = logits2d.shape[-1]
    nv = vvalid or V
    z = logits2d.float()[:, :nv]
    m = z.max(-1).values
    e = torch.exp(z - m[:, None])
    loc = target - vstart
    inr = (loc >= 0) & (loc < nv)
    t = torch.where(inr, z.gather(1, loc.clamp(0, nv - 1)[:, None])[:, 0], torch.zeros_like(m))
    out = torch.zeros(logits2d.shape, dtype=torch.float32, device=logits2d.device)
    out[:, :nv] = e
    logits2d.copy_(out.to(logits2d.dtype))
    return torch.stack([m, e.sum(-1), t])


def combine_ce_stats(allst, st, t, ignore_index):
    """Per-row loss and softmax scale c from every rank's ``ce_local_pass`` statistics
    ``allst`` [ranks, 3, rows] (this rank's: ``st``): M = max m_r, S = sum s_r exp(m_r - M),
    loss = log S + M - x_t, c = exp(m_mine - M) / S (0 for ignored rows)."""
    M = allst[:, 0].max(0).values
    S = (allst[:, 1] * torch.exp(allst[:, 0] - M)).sum(0)
    ign = t == ignore_index
    loss = torch.where(ign, torch.zeros_like(S), torch.log(S) + M - allst[:, 2].sum(0))
    c = torch.where(ign, torch.zeros_like(S), torch.exp(st[0] - M) / S)
    return loss, c


def subtract_onehot_(l2, t, c, vstart, vvalid, ignore_index):
    """The one-hot at ONE element per row whose target lies in this slice: e[t] -= 1 / c, so that
    c e = softmax - onehot. No host sync (every row writes its clamped position; rows without an
    in-slice target write their own value back)."""
    V = l2.shape[-1]
    loc = t - vstart
    inr = (loc >= 0) & (loc < (vvalid or V)) & (t != ignore_index)
    lin = torch.arange(l2.shape[0], device=l2.device) * V + loc.clamp(0, V - 1)
    flat = l2.view(-1)
    cur = flat[lin].float()
    flat[lin] = torch.where(inr, cur - 1.0 / c, cur).to(flat.dtype)


class VocabParallelLMHeadCE(torch.autograd.Function):
    """LM head + CE for a vocabulary split over the TP group (TP > 1), the LM-head GEMM and the loss
    as ONE op with a single pass over this rank's [tokens, V / tp] logits (the
    TP = 1 form is ``LMHeadCrossEntropy``). Same math as Megatron's parallel_lm_logits +
    vocab-parallel CE (/root/reference/3_training_megatron-lm/pretrain_gpt.py:51-57;
    megatron/arguments.py:992-994):

    * logits = X W_r^T — with sequence parallelism through the ring all-gather collective-matmul
      (``_ColumnSPLinear``'s forward);
    * ``ce_local_pass`` overwrites them with e = exp(x - m_r) and returns (m_r, s_r, x_t) per row;
    * ONE all-gather of those [3, tokens] statistics replaces the three all-reduces (MAX, SUM,
      SUM): M = max m_r, S = sum s_r exp(m_r - M), loss = log S + M - x_t;
    * with the row scale c = exp(m_r - M) / S, softmax = c e, so the one-hot is subtracted at ONE
      element per row: e[t] -= 1 / c (no second pass);
    * backward: D = c e - onehot never exists — the per-row c dloss goes on the [tokens, hidden]
      side: dX = diag(c dl) (E W) (reduce-scattered along the sequence by the ring, or all-reduced
      without SP) and dW = E^T diag(c dl) X.

    Against logits -> separate stats kernel -> 3 all-reduces -> backward kernel over the logits,
    this drops one full read of the logits per micro-batch on the last pipeline stage.
    bf16 only (the hidden-side scaling, see ``lm_head_ce_ok``)."""

    @staticmethod
    def forward(ctx, x, weight, target, ignore_index, vstart, vvalid, sp):
        group = _tp_group()
        ws = dist.get_world_size(group)
        x = x.contiguous()
        if sp:
            n = x.shape[0]
            logits = x.new_empty((n * ws,) + tuple(x.shape[1:-1]) + (weight.shape[0],))
            total = ag_ring(x, group, lambda lo, ch: _mm_into(logits[lo:lo + ch.shape[0]], ch, weight))
        else:
            n = x.shape[0] // ws
            total = x
            logits = linear_rows(x, weight)
        V = logits.shape[-1]
        l2 = logits.view(-1, V)
        t = target.contiguous().view(-1)
        st = ce_local_pass(l2, t, vstart, vvalid).contiguous()
        allst = st.new_empty((ws,) + tuple(st.shape))
        if ws > 1:
            from ..comm import stats as _cs
            with _cs.blocking("all_gather", group, allst.numel() * allst.element_size()):
                dist.all_gather_into_tensor(allst.view(-1), st.view(-1), group=group)
        else:
            allst[0].copy_(st)
        loss, c = combine_ce_stats(allst, st, t, ignore_index)
        subtract_onehot_(l2, t, c, vstart, vvalid, ignore_index)
        ctx.save_for_backward(total, weight, logits, c)
        ctx.sp, ctx.n = sp, n
        return loss.view(target.shape)

    @staticmethod
    def backward(ctx, dloss):
        total, weight, e, c = ctx.saved_tensors
        group = _tp_group()
        n = ctx.n
        r = dloss.contiguous().view(-1).float() * c          # per-row scale of E = c dl
        r3 = r.view(e.shape[:-1] + (1,))
        wt = _dgrad_weight_t(weight)
        res = {}

        def wgrad():
            H = total.shape[-1]
            hs = torch.mul(total.reshape(-1, H), r.view(-1, 1)).to(total.dtype)
            res["dw"] = _wgrad(weight, e.view(-1, e.shape[-1]), hs)
            _flush_wgrad()

        def part(lo, m, o):
            g = _dgrad_rows(e[lo:lo + m], weight, wt, o)
            g.mul_(r3[lo:lo + m])
            return g
        if ctx.sp:
            gi = rs_ring(part, group, e.shape[:-1] + (weight.shape[1],), e, wgrad)
        else:
            gi = dgrad(e, weight, wt)
            gi.mul_(r3)
            h = dist.all_reduce(gi, group=group, async_op=True) if dist.get_world_size(group) > 1 else None
            wgrad()
            if h is not None:
                h.wait()
        if "dw" not in res:
            wgrad()
        return gi, res["dw"], None, None, None, None, None


def vp_lm_head_ce_ok(h, weight, tp: int) -> bool:
    """Whether ``VocabParallelLMHeadCE`` applies: TP > 1, HIP kernels on and bf16 operands (or the
    CPU reference with SMDT_LM_HEAD_CE_CPU=1, for the Gloo equivalence tests), a vocab slice whose
    row fits one block's registers (V / tp % 8 == 0, <= 65536). SMDT_LM_HEAD_CE=0 disables."""
    from ..ops import _ext
    if not (_LM_HEAD_CE and tp > 1 and weight.shape[0] % 8 == 0 and weight.shape[0] <= 65536
            and weight.dtype == h.dtype):
        return False
    if h.is_cuda:
        return _ext.use_kernels(h) and h.dtype == torch.bfloat16
    return os.environ.get("SMDT_LM_HEAD_CE_CPU", "0") == "1"


def _ext_mod():
    from ..ops import _ext
    return _ext.ext()


def lm_head_ce_ok(h, weight, tp: int) -> bool:
    """Whether ``LMHeadCrossEntropy`` applies: HIP kernels on, TP = 1, bf16 operands, a vocab
    whose row fits one block's registers (V % 8 == 0, V <= 65536). SMDT_LM_HEAD_CE=0 disables.

    bf16 only: the backward scales the hidden rows by the per-token dloss (``h * dl`` stored in
    the 16-bit type). Under an fp16 loss scale dl ~ scale / tokens, and |h| > 1 would overflow
    fp16 at loss scales the separate CE path (dl times softmax - onehot, |.| <= 1) still takes."""
    from ..ops import _ext
    return (_LM_HEAD_CE and tp == 1 and _ext.use_kernels(h) and h.dtype == torch.bfloat16
            and weight.dtype == h.dtype and weight.shape[0] % 8 == 0 and weight.shape[0] <= 65536)


_LM_HEAD_CE = os.environ.get("SMDT_LM_HEAD_CE", "1") == "1"


def linear_with_grad_accumulation_and_async_allreduce(x, weight, bias, sequence_parallel=False,
                                                      async_grad_allreduce=False, add_bias=True):
    if sequence_parallel and _TP_OVERLAP and _tp_size() > 1:
        return _ColumnSPLinear.apply(x, weight, bias, add_bias)
    return LinearWithGradAccumulationAndAsyncCommunication.apply(x, weight, bias, sequence_parallel,
                                                                 async_grad_allreduce, add_bias)


# --------------------------------------------------------------------------------------------
# Sequence-parallel linears with the TP collective fused into the GEMM as a ring (collective
# matmul): the all-gather / reduce-scatter moves one sequence chunk per step over RCCL p2p while
# the GEMM of the previous / next chunk runs, instead of a monolithic collective followed by a
# monolithic GEMM. On MI355X the TP pair talks over ONE xGMI link (~64-77 GB/s per direction),
# which at GPT-2 345M shapes moves a layer's activations slower than the MFMA cores consume them,
# so every byte in flight must have a GEMM beside it. Backward collectives additionally drain the
# deferred weight-gradient queue before they are waited for (Megatron's "launch dgrad collective
# -> wgrad GEMM -> wait", arguments.py:837-842, with the grouped MFMA wgrad as the overlapped work).

_TP_OVERLAP = os.environ.get("SMDT_TP_OVERLAP", "1") == "1"
_LB_RING_ASYNC = os.environ.get("SMDT_LOOPBACK_RING_ASYNC", "0") == "1"


def _ring(group):
    ws = dist.get_world_size(group)
    r = dist.get_rank(group)
    ranks = dist.get_process_group_ranks(group)
    return ws, r, ranks[(r + 1) % ws], ranks[(r - 1) % ws]


def _exchange(send, recv, nxt, prv, group):
    """One ring step: send to next and receive from prev in ONE p2p group (matched per peer in
    issue order, so a 2-rank ring with next == prev cannot deadlock). A 2-rank ring on an
    MI355X node goes over every xGMI link through the relay engine (comm/relay.py) when one was
    built for ``group`` and measured faster than RCCL's single-link p2p."""
    if _lb.is_loopback(group):
        # single-process TP emulation: the transfer as a local copy on the compute stream (issuing
        # it on the loopback side stream, as the real exchange runs beside the chunk GEMM, measured
        # SLOWER: 202.4 -> 219.7 ms per stage-1 rank, the per-exchange stream hand-offs cost more
        # than the overlap gains; profiles/r4_loopback_ring_async_neg/). SMDT_LOOPBACK_RING_ASYNC=1
        # re-runs that arm (the side stream is now a high-priority one).
        standin = _lb.link_standin() if send.is_cuda else None
        if standin is not None:
            # paced link stand-in (SMDT_LINK_STANDIN): the modelled link time and the relay's CU
            # footprint, on the side stream beside the rank's compute, waited for like the relay
            gbps, blocks = standin
            ns = int(_nbytes(send) / gbps)          # bytes / (GB/s) = ns
            C = _ext.ext()
            SPLIT_STATS["standin_exchanges"] = SPLIT_STATS.get("standin_exchanges", 0) + 1
            works = [group._issue([send, recv], lambda: C.paced_copy(recv, send, blocks, ns), [recv])]
            _hold_cus(works, blocks)
            return works
        if _LB_RING_ASYNC and send.is_cuda:
            return [group._issue([send, recv], lambda: recv.copy_(send), [recv])]
        recv.copy_(send)
        return []
    if nxt == prv:
        eng = _relay.engine_for(group)
        if eng is not None:
            h = eng.exchange_async(send, recv)
            if h is not None:
                _cs.collective("p2p", group, _nbytes(send), transport="relay", events=h.timing())
                _hold_cus([h], eng.cu_blocks())
                return [h]
    if send.is_cuda and dist.get_backend(group) == "gloo":
        # Gloo rehearsals with CUDA tensors (several ranks on one GPU, SMDT_BENCH_BACKEND=gloo):
        # a rank that sends to and receives from the same peer at once never completes its
        # receive (both ranks of a tp2 ring stalled in the first wait, profiles/r4_rehearse_tp2/);
        # the exchange goes through host buffers, synchronously. RCCL runs never take this path.
        s_cpu = send.detach().cpu()
        r_cpu = torch.empty(recv.shape, dtype=recv.dtype)
        for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, s_cpu, nxt, group),
                                         dist.P2POp(dist.irecv, r_cpu, prv, group)]):
            w.wait()
        recv.copy_(r_cpu)
        return []
    works = dist.batch_isend_irecv([dist.P2POp(dist.isend, send, nxt, group),
                                    dist.P2POp(dist.irecv, recv, prv, group)])
    _cs.collective("p2p", group, _nbytes(send), work=works[0] if len(works) == 1 else None)
    return works


def _linear_into(x, w, out=None):
    """x W^T into ``out`` (returned) when given, else a new tensor (``rs_ring`` partials)."""
    if out is None and _RING_GEMM_TN and _CU_HELD and x.is_cuda:
        out = x.new_empty(tuple(x.shape[:-1]) + (w.shape[0],))
    if out is None:
        return torch.nn.functional.linear(x, w)
    _mm_into(out, x, w)
    return out


def _dgrad_rows(g, weight, wt, out=None):
    """dX = g @ weight into ``out`` (returned) when given, else a new tensor."""
    if out is None:
        return dgrad(g, weight, wt)
    dgrad_into(out, g, weight, wt)
    return out


# SMDT_RING_GEMM_TN=1: ring-chunk GEMMs issued while an exchange holds CUs run on gemm_tn with
# the leftover grid (gemm_tn_blocks) instead of hipBLASLt, whose full-chip grid races the exchange
_RING_GEMM_TN = os.environ.get("SMDT_RING_GEMM_TN", "0") == "1"


def _mm_into(dst, a, w, bias=None):
    """dst[..., o] = a[..., k] @ w[o, k]^T (+ bias) written in place (hipBLASLt out= GEMM)."""
    a2 = a.reshape(-1, a.shape[-1])
    d2 = dst.view(-1, dst.shape[-1])
    if _RING_GEMM_TN and _CU_HELD and a2.is_cuda and a2.is_contiguous() and d2.is_contiguous() \
            and a2.dtype in (torch.bfloat16, torch.float16) and w.dtype == a2.dtype \
            and (bias is None or bias.dtype == a2.dtype) and _ext.ext().gemm_tn_supported(a2, w) \
            and (a2.shape[0] // 256) * (w.shape[0] // 256) >= gemm_tn_blocks():
        # (only when the GEMM has a tile for every CU it may use: GPT-3 tp4's 2,048-row chunks have
        # 128 and stay on hipBLASLt, profiles/r6_mix/)
        _ext.ext().gemm_tn(a2, w, 1 if bias is not None else 0, bias, d2, None, gemm_tn_blocks())
        return
    if bias is not None:
        torch.addmm(bias, a2, w.t(), out=d2)
    else:
        torch.mm(a2, w.t(), out=d2)


def _direct(group):
    """The multi-link TP exchange engine (comm/tp_direct.py) bound to ``group``, or None."""
    st = ps.get_state()
    td = getattr(st, "tp_direct", None)
    return td if (td is not None and group is st.tp_group and td.active) else None


_SP_GATHER_SLOTS = os.environ.get("SMDT_SP_GATHER_SLOTS", "1") == "1"   # A/B switch
# ring all-gathers whose local block was already in place (written by its producer) vs copied
AG_RING_STATS = {"in_place": 0, "copied": 0}


def _gather_buffer(x, ws, r):
    """The [n * ws, ...] all-gather buffer of ``x`` with x in slot r: the buffer x's producer wrote
    it into (the norm's gather slot, no copy) or a new one with x copied in."""
    n = x.shape[0]
    mark = getattr(x, "_smdt_gather", None)
    if (mark is not None and mark[1] == r and mark[0].shape[0] == n * ws and mark[0].shape[1:] == x.shape[1:]
            and mark[0].is_contiguous() and x.is_contiguous() and x.data_ptr() == mark[0][r * n].data_ptr()):
        AG_RING_STATS["in_place"] += 1
        return mark[0]
    total = x.new_empty((n * ws,) + tuple(x.shape[1:]))
    total[r * n:(r + 1) * n].copy_(x)
    AG_RING_STATS["copied"] += 1
    return total


# Sub-batch interleave (``models/transformer.ParallelTransformer``, SMDT_SP_SUBBATCH): the two
# halves of a micro-batch run each layer phase by phase, alternately, so one half's TP-pair
# exchange travels beside the other half's GEMMs / attention instead of beside half of its own
# GEMM only (a 2-rank ring's sole overlap partner in forward: profiles/r5_predict_tp2x/). The
# issue order of the exchanges stays a pure function of the layer stack on both partners, which
# the relay's per-call epochs need. Forward only: the backward's exchanges already overlap the
# drained weight-gradient GEMMs.
_SPLIT = {"on": False}
# Forward reduce-scatters whose consumer is a fused norm (``defer_rs_add``, set by the layer
# stack): the 2-rank ring's combine (own partial + the peer's) is left to the norm kernel, which
# reads both summands (ops/functional.bias_dropout_add_norm, x2) instead of a separate add pass.
_DEFER_ADD = {"on": False}
_DEFER_RS_ADD = os.environ.get("SMDT_DEFER_RS_ADD", "1") == "1"


class defer_rs_add:
    """Context: forward ring reduce-scatters leave their combine to the consuming fused norm."""

    def __enter__(self):
        self.prev = _DEFER_ADD["on"]
        _DEFER_ADD["on"] = _DEFER_RS_ADD
        return self

    def __exit__(self, *exc):
        _DEFER_ADD["on"] = self.prev
        return False


def _bwd_add_to_norm(x) -> bool:
    """Whether a column SP linear's backward reduce-scatter may leave its combine to x's producer:
    inside the layer stack (``defer_rs_add``), x written by the fused norm kernel into its
    all-gather slot (``_smdt_gather``: the norm's autograd node receives the gradient as is) and on
    the kernel path (the norm backward that reads the pending summand)."""
    return (_DEFER_ADD["on"] and not _SPLIT["on"] and getattr(x, "_smdt_gather", None) is not None
            and _ext.use_kernels(x))


# Ledger of the pending summands: every summand hung on a tensor by
# ``set_pending_add`` must be taken by ``take_pending_add`` (the fused norm, forward or backward,
# or ``materialize_add``). A consumer that reads the tensor some other way would silently miss the
# peer's half, so anything left over at a check point raises instead: the end of the layer
# stack's forward and the end of its backward (models/transformer.ParallelTransformer), and
# DistributedDataParallel.finish_grad_sync.
_ADD_LEDGER = {"issued": 0, "consumed": 0, "live": {}}


# Forward guard (SMDT_DEFER_RS_GUARD, default on): a row-parallel output whose combine is deferred
# becomes a ``PendingPartial`` — its class is swapped in place (0.5 us; an ``as_subclass`` alias
# cost 6 us, +1.5 ms per emulated N = 8 stage step, profiles/r6_guard/) to a tensor subclass
# whose every torch operation raises, apart from metadata reads — until its fused norm takes the
# summand (``take_pending_add``) and turns it back into a plain tensor (``plain``). A consumer
# that reads it before that (a forward hook, a model variant reading the output twice or through
# a non-fused norm) fails at its first read instead of seeing a partial sum.
_GUARD = os.environ.get("SMDT_DEFER_RS_GUARD", "1") == "1"


def _meta_funcs():
    T = torch.Tensor
    out = {T.as_subclass, T.data_ptr, T.dim, T.size, T.numel, T.element_size, T.stride, T.is_contiguous,
           T.__len__, T.__hash__}
    for name in ("shape", "dtype", "device", "is_cuda", "requires_grad", "grad_fn", "ndim", "layout",
                 "is_leaf", "_version", "names"):
        prop = getattr(T, name, None)
        if prop is not None and hasattr(prop, "__get__"):
            out.add(prop.__get__)
    return out


class PendingPartial(torch.Tensor):
    """See _GUARD. Only metadata reads and ``as_subclass`` pass."""

    _META = None

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        if cls._META is None:
            cls._META = _meta_funcs()
        if func in cls._META:
            with torch._C.DisableTorchFunctionSubclass():
                return func(*args, **(kwargs or {}))
        name = getattr(func, "__name__", str(func))
        raise RuntimeError(
            f"a row-parallel output whose reduce-scatter combine was deferred to its fused norm was "
            f"read by another consumer ({name}) — it holds only this rank's partial sum. Run with "
            "SMDT_DEFER_RS_ADD=0, or keep the fused norm as the only consumer.")


def plain(t):
    """``t`` as a plain tensor again (a ``PendingPartial``'s class is swapped back in place)."""
    if type(t) is PendingPartial:
        t.__class__ = torch.Tensor
    return t


def set_pending_add(t, x2, where: str):
    """Hang ``x2`` on ``t`` for its consumer; returns t (forward outputs: turned into a
    ``PendingPartial`` in place under the guard)."""
    if _GUARD and where == "forward output" and type(t) is torch.Tensor:
        t.__class__ = PendingPartial
    t._smdt_add = x2
    _ADD_LEDGER["issued"] += 1
    _ADD_LEDGER["live"][id(t)] = where
    return t


def take_pending_add(t):
    """The pending summand of ``t`` (removed from it and from the ledger), or None. The caller
    then reads ``plain(t)``."""
    x2 = getattr(t, "_smdt_add", None)
    if x2 is not None:
        del t._smdt_add
        _ADD_LEDGER["consumed"] += 1
        _ADD_LEDGER["live"].pop(id(t), None)
    return x2


def check_pending_adds(where: str):
    """Raise if a deferred reduce-scatter summand was issued but never consumed. (Also drops any CU
    hold left by an exchange no ring waited for: every TP exchange of a layer-stack pass is
    complete at these check points.)"""
    _CU_HELD.clear()
    live = _ADD_LEDGER["live"]
    if live:
        kinds = sorted(set(live.values()))
        n = len(live)
        live.clear()
        raise RuntimeError(
            f"{n} deferred reduce-scatter summand(s) ({', '.join(kinds)}) were never added by their "
            f"consumer (checked at {where}): a hook, a second consumer or a non-fused norm read a "
            "row-parallel output / column-parallel input gradient without the peer's partial. Run "
            "with SMDT_DEFER_RS_ADD=0 or keep the fused norm as the only consumer.")


def foreign_hooks(module) -> bool:
    """Whether any hook other than the framework's own parameter-wait pre-hooks (marked
    ``_smdt_internal``) could see the layer stack's activations or gradients: global module hooks,
    or forward / backward hooks on ``module`` or a submodule. Deferring the reduce-scatter combine
    is only safe without them (a hook would read a tensor missing the peer's partial)."""
    from torch.nn.modules import module as _M
    for name in ("_global_forward_hooks", "_global_forward_pre_hooks", "_global_backward_hooks",
                 "_global_backward_pre_hooks"):
        if getattr(_M, name, None):
            return True
    for m in module.modules():
        if m._forward_hooks or m._backward_hooks or getattr(m, "_backward_pre_hooks", None):
            return True
        for h in m._forward_pre_hooks.values():
            if not getattr(h, "_smdt_internal", False):
                return True
    return False


def materialize_add(t):
    """Apply a pending reduce-scatter summand (``defer_rs_add``) in place; returns the plain t."""
    x2 = take_pending_add(t)
    t = plain(t)
    if x2 is not None:
        t.data.add_(x2)
    return t
_AG_PENDING = {}      # (data_ptr, shape) of a started all-gather's input -> (total, works, rank, n)
_RS_PENDING = []      # outputs whose reduce-scatter was started but not yet combined
SPLIT_STATS = {"ag_started": 0, "rs_deferred": 0, "rs_add_to_norm": 0, "bwd_add_to_norm": 0}


def _pending_key(x):
    return (x.data_ptr(), tuple(x.shape)) if _AG_PENDING else None


def subbatch_capable(st) -> bool:
    """Whether the TP exchanges can be started / left in flight for the sub-batch interleave: a
    2-rank ring writing into producer-filled gather slots, or a TP4 / TP8 direct engine."""
    if st.tp == 2:
        return sp_gather_spec() is not None
    return st.tp in (4, 8) and _direct(st.tp_group) is not None


def ag_start(x, group):
    """Issue the 2-rank ring all-gather of ``x`` now (TP4 / TP8: the direct engine's whole-chunk
    gather); the ``ag_ring`` call of x's consumer then waits and runs ONE GEMM over all chunks
    (the ring: its local chunk's GEMM, the wait, the peer's chunk)."""
    td = _direct(group)
    if td is not None:
        started = td.start_all_gather(x)
        if started is not None:     # (world-uniform: else the consumer's ag_ring gathers as usual)
            total, hs = started
            _AG_PENDING[(x.data_ptr(), tuple(x.shape))] = (total, hs, td.rank, x.shape[0])
            SPLIT_STATS["ag_started"] += 1
        return x
    ws, r, nxt, prv = _ring(group)
    assert ws == 2, "ag_start: 2-rank rings only"
    x = x.contiguous()
    n = x.shape[0]
    total = _gather_buffer(x, ws, r)
    peer = 1 - r
    # the receive goes through ``.data`` (same storage, own version counter): x is usually a view
    # of ``total`` returned by the fused norm (a multi-output autograd node), and an in-place write
    # into its base seen by autograd before x's consumer is applied would be refused
    raw = total.data
    works = _exchange(raw[r * n:(r + 1) * n], raw[peer * n:(peer + 1) * n], nxt, prv, group)
    _AG_PENDING[(x.data_ptr(), tuple(x.shape))] = (total, works, r, n)
    SPLIT_STATS["ag_started"] += 1
    return x


def rs_finish(t):
    """Complete a reduce-scatter ``rs_ring`` left in flight under the sub-batch interleave: wait for
    the peer's partial of this rank's chunk and add it into ``t`` (in place, outside autograd: the
    gradient of the sum is the gradient of t). Returns t; a no-op for any other tensor."""
    pend = getattr(t, "_smdt_rs_pending", None)
    if pend is None:
        return t
    del t._smdt_rs_pending
    works, incoming, _keep, group = pend
    _wait_works(works, group)
    if incoming is not None:     # the ring's combine (the direct engine's output is the sum)
        t.data.add_(incoming)    # outside autograd (t may be a view output of the linear's Function)
    try:
        _RS_PENDING.remove(t)
    except ValueError:
        pass
    return t


def begin_subbatch():
    _SPLIT["on"] = True


class PendingAddCheck(torch.autograd.Function):
    """Identity on the layer stack's input whose backward (the last node of the stack's backward)
    checks that every deferred summand of that backward was consumed (``check_pending_adds``)."""

    @staticmethod
    def forward(ctx, x):
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        check_pending_adds("the end of the layer stack's backward")
        return g


class WgradMergeScope(torch.autograd.Function):
    """Identity whose backward sets ``DEFERRED_WGRAD.merge_repeats`` to ``on``. The sub-batch
    interleave wraps its output with on=True (the first node of the pass's backward) and its
    input with on=False (the last), so the merge of the two halves' pushes is scoped to that
    backward and every later pass flushes repeated pushes in order again."""

    @staticmethod
    def forward(ctx, x, on):
        ctx.on = bool(on)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        DEFERRED_WGRAD.merge_repeats = ctx.on
        return g, None


def end_subbatch():
    """Leave the interleave: any exchange still in flight is completed (a consumer that never came
    would otherwise leave the relay's epochs of the two partners apart)."""
    _SPLIT["on"] = False
    for t in list(_RS_PENDING):
        rs_finish(t)
    _RS_PENDING.clear()
    for total, works, _r, _n in list(_AG_PENDING.values()):
        for w in works:
            w.wait()
    _AG_PENDING.clear()
    _CU_HELD.clear()


# SMDT_RING_PIECES=k (2-rank rings): each exchange goes out in k row pieces, so the peer chunk's
# GEMM starts on the first piece (all-gather) and the first partial piece leaves before the whole
# partial exists (reduce-scatter); pieces keep whole 256-row GEMM blocks (else one piece)
_RING_PIECES = int(os.environ.get("SMDT_RING_PIECES", "1") or 1)


def _row_pieces(n: int, rows_per: int, k: int, align: int = 256):
    """[(a, b)) bounds of k row pieces of an n-row chunk (dim 0) whose GEMM rows (x rows_per) stay
    multiples of ``align`` (256 on the GPU: gemm_tn's row blocks); [(0, n)] when impossible."""
    if k <= 1 or n % k:
        return [(0, n)]
    step = n // k
    if (step * rows_per) % align:
        return [(0, n)]
    return [(i * step, (i + 1) * step) for i in range(k)]


def ag_ring(x, group, chunk_fn=None, before_last_wait=None, _skip_direct=False, bulk=False):
    """All-gather ``x`` along dim 0 over ``group`` as a ring; ``chunk_fn(lo, rows)`` runs on the
    gathered rows [lo, lo + rows.shape[0]) (dim 0) as soon as they are resident, while the next
    chunk is in flight: the ring hands over whole chunks (lo = c * n). Returns the gathered tensor.
    TP groups of 4 / 8 with a direct engine (comm/tp_direct.py) gather over all of the group's
    links at once instead, in row pieces: the local chunk's GEMM beside the first piece, every
    peer's rows of piece j as soon as piece j has landed."""
    pend = _AG_PENDING.pop(_pending_key(x), None)
    if pend is not None:
        # started earlier by ``ag_start`` (sub-batch interleave): the other half's phase ran beside
        # the transfer, so the consumer waits and runs ONE GEMM over both chunks (16,384 rows at
        # the BASELINE point instead of two 8,192-row chunk GEMMs)
        total, works, r, n = pend
        if before_last_wait is not None:
            before_last_wait()
        _wait_works(works, group)
        if chunk_fn is not None:
            chunk_fn(0, total)
        return total
    td = None if _skip_direct else _direct(group)
    if td is not None:
        out = td.all_gather(x, chunk_fn, before_last_wait)
        if out is not None:
            _cs.collective("all_gather", group, _nbytes(out), transport="xgmi")
            return out
    ws, r, nxt, prv = _ring(group)
    n = x.shape[0]
    total = _gather_buffer(x, ws, r)
    if bulk and ws == 2:
        # a sub-batch half's backward (``bulk``): the exchange beside the drained weight-gradient
        # GEMMs, then ONE GEMM over both chunks (half-size chunk GEMMs measured slow)
        peer = 1 - r
        works = _exchange(total[r * n:(r + 1) * n], total[peer * n:(peer + 1) * n], nxt, prv, group)
        if before_last_wait is not None:
            before_last_wait()
        _wait_works(works, group)
        if chunk_fn is not None:
            chunk_fn(0, total)
        return total
    rows_per = x.numel() // max(x.shape[0], 1) // max(x.shape[-1], 1)
    bounds = _row_pieces(n, rows_per, _RING_PIECES, 256 if x.is_cuda else 1) if ws == 2 else [(0, n)]
    if len(bounds) > 1:
        # 2-rank ring in row pieces: every piece of this rank's chunk goes out at once (the
        # engine's stream runs them in order), the local chunk's GEMM runs beside them, then each
        # peer piece's GEMM as soon as that piece has landed
        peer = 1 - r
        works_j = [_exchange(total[r * n + a:r * n + b], total[peer * n + a:peer * n + b], nxt, prv, group)
                   for a, b in bounds]
        SPLIT_STATS["ring_pieces"] = SPLIT_STATS.get("ring_pieces", 0) + len(bounds)
        if chunk_fn is not None:
            chunk_fn(r * n, x)
        for j, (a, b) in enumerate(bounds):
            if j == len(bounds) - 1 and before_last_wait is not None:
                before_last_wait()
            fill_exchange_wait()
            _wait_works(works_j[j], group)
            if chunk_fn is not None:
                chunk_fn(peer * n + a, total[peer * n + a:peer * n + b])
        return total
    for s in range(ws):
        c = (r - s) % ws
        works = None
        if s < ws - 1:
            nc = (c - 1) % ws
            works = _exchange(total[c * n:(c + 1) * n], total[nc * n:(nc + 1) * n], nxt, prv, group)
        if chunk_fn is not None:
            chunk_fn(c * n, x if s == 0 else total[c * n:(c + 1) * n])
        if works is not None:
            if s == ws - 2 and before_last_wait is not None:
                before_last_wait()
            fill_exchange_wait()
            _wait_works(works, group)
    return total


def rs_ring(partial_fn, group, full_shape, ref, before_last_wait=None, bulk=False, defer_add=False):
    """Reduce-scatter along dim 0 over ``group`` as a ring. The tensor being reduced (``full_shape``,
    ``ref``'s dtype / device) is produced on demand: ``partial_fn(lo, rows, out)`` computes its rows
    [lo, lo + rows) — a GEMM on those rows — into ``out`` when given (and returns it), else into a
    new tensor. Ring step s computes the next chunk's partial while the previous one is in flight.
    Returns this rank's reduced chunk. TP groups of 4 / 8 with a direct engine write the partials
    straight into the engine's input buffer in row pieces, each piece reduce-scattered over every
    link of the group while the next piece's GEMMs run."""
    td = _direct(group)
    if td is not None and _SPLIT["on"] and before_last_wait is None:
        # sub-batch interleave: every chunk's partial in ONE GEMM, the reduce-scatter left in
        # flight (``rs_finish`` waits) while the other half's phase runs
        n = full_shape[0] // td.world
        full = partial_fn(0, td.world * n, None)
        started = td.start_reduce_scatter(full)
        if started is None:
            out = full.new_empty((n,) + tuple(full.shape[1:]))
            dist.reduce_scatter_tensor(out, full.contiguous(), group=group)
            return out
        out, hs = started
        out._smdt_rs_pending = (hs, None, full, group)
        _RS_PENDING.append(out)
        SPLIT_STATS["rs_deferred"] += 1
        _cs.collective("reduce_scatter", group, _nbytes(out) * td.world, transport="xgmi")
        return out
    if td is not None:
        out = td.reduce_scatter(partial_fn, full_shape, ref, before_last_wait)
        _cs.collective("reduce_scatter", group, _nbytes(out) * td.world, transport="xgmi")
        return out
    ws, r, nxt, prv = _ring(group)
    n = full_shape[0] // ws
    if _SPLIT["on"] and ws == 2 and before_last_wait is None:
        # sub-batch interleave: the peer's partial, its exchange, this rank's partial; the combine
        # is left to ``rs_finish`` so the other half's work runs while the partial travels
        # (one GEMM over both chunks, then the peer's half goes out; ``own`` is a view of it)
        peer = 1 - r
        full = partial_fn(0, 2 * n, None)
        part = full[peer * n:(peer + 1) * n]
        incoming = torch.empty_like(part)
        works = _exchange(part, incoming, nxt, prv, group)
        own = full[r * n:(r + 1) * n]
        own._smdt_rs_pending = (works, incoming, full, group)
        _RS_PENDING.append(own)
        SPLIT_STATS["rs_deferred"] += 1
        return own
    if bulk and ws == 2:
        # a sub-batch half's backward: one GEMM over both chunks, the peer's half out beside the
        # drained weight-gradient GEMMs, then the combine
        peer = 1 - r
        full = partial_fn(0, 2 * n, None)
        incoming = torch.empty_like(full[:n])
        works = _exchange(full[peer * n:(peer + 1) * n], incoming, nxt, prv, group)
        if before_last_wait is not None:
            before_last_wait()
        _wait_works(works, group)
        return full[r * n:(r + 1) * n].add_(incoming)
    rows_per = 1
    for d in full_shape[1:-1]:
        rows_per *= d
    bounds = _row_pieces(n, rows_per, _RING_PIECES, 256 if ref.is_cuda else 1) if ws == 2 else [(0, n)]
    if len(bounds) > 1:
        # 2-rank ring in row pieces: the peer's partial piece by piece, each piece out as soon as
        # it exists, then this rank's own partial beside the transfers, then the combine
        peer = 1 - r
        incoming = None
        works_j, keep = [], []
        for a, b in bounds:
            part = partial_fn(peer * n + a, b - a, None)
            if incoming is None:
                incoming = torch.empty((n,) + tuple(part.shape[1:]), dtype=part.dtype, device=part.device)
            keep.append(part)
            works_j.append(_exchange(part, incoming[a:b], nxt, prv, group))
        SPLIT_STATS["ring_pieces"] = SPLIT_STATS.get("ring_pieces", 0) + len(bounds)
        own = partial_fn(r * n, n, None)
        for j in range(len(bounds)):
            if j == len(bounds) - 1 and before_last_wait is not None:
                before_last_wait()
            fill_exchange_wait()
            _wait_works(works_j[j], group)
        if (_DEFER_ADD["on"] and before_last_wait is None) or defer_add:
            own = set_pending_add(own, incoming, "backward dgrad" if defer_add else "forward output")
            SPLIT_STATS["bwd_add_to_norm" if defer_add else "rs_add_to_norm"] += 1
            return own
        return own.add_(incoming)
    works, incoming, keep = None, None, []
    for s in range(ws):
        c = (r - s - 1) % ws
        part = partial_fn(c * n, n, None)
        if works is not None:
            if s == ws - 1 and before_last_wait is not None:
                before_last_wait()
            fill_exchange_wait()
            _wait_works(works, group)
            if s == ws - 1 and ws == 2 and ((_DEFER_ADD["on"] and before_last_wait is None) or defer_add):
                # the consuming norm adds it (see _DEFER_ADD)
                part = set_pending_add(part, incoming, "backward dgrad" if defer_add else "forward output")
                SPLIT_STATS["bwd_add_to_norm" if defer_add else "rs_add_to_norm"] += 1
                return part
            part = part.add_(incoming)
        if s == ws - 1:
            return part
        incoming = torch.empty_like(part)
        keep.append(part)
        works = _exchange(part, incoming, nxt, prv, group)
    return None  # unreachable


def sp_gather_spec():
    """(world, rank) of the TP group when sequence-parallel linears run the ring collective-matmul
    (``ag_ring`` can take a producer-filled gather buffer), else None. The multi-link direct
    engine allocates its own buffers."""
    st = ps.get_state()
    if not _TP_OVERLAP or not _SP_GATHER_SLOTS or st.tp <= 1 or st.tp_group is None:
        return None
    td = getattr(st, "tp_direct", None)
    if td is not None and td.active:
        return None
    return st.tp, st.tp_rank


def _flush_wgrad():
    DEFERRED_WGRAD.flush_opportunistic()


class _ColumnSPLinear(torch.autograd.Function):
    """Column-parallel linear on a sequence-parallel input: forward = ring all-gather fused with
    the GEMM (the gathered input is kept for the weight gradient: 288 GB of HBM makes the
    backward re-gather unnecessary); backward = dgrad GEMM fused with a ring reduce-scatter, the
    weight gradient queued and drained while the last chunk is in flight."""

    @staticmethod
    def forward(ctx, x, weight, bias, add_bias=True):
        group = _tp_group()
        x = x.contiguous()
        n = x.shape[0]
        ws = dist.get_world_size(group)
        out = x.new_empty((n * ws,) + tuple(x.shape[1:-1]) + (weight.shape[0],))
        fb = bias if add_bias else None
        total = ag_ring(x, group, lambda lo, ch: _mm_into(out[lo:lo + ch.shape[0]], ch, weight, fb))
        ctx.save_for_backward(total, weight)
        ctx.bias_p = bias
        ctx.n = n
        ctx.bulk = _SPLIT["on"]
        ctx.defer_add = _bwd_add_to_norm(x)
        return out

    @staticmethod
    def backward(ctx, g):
        total, weight = ctx.saved_tensors
        group = _tp_group()
        g = g.contiguous()
        n = ctx.n
        res = {}

        def wgrad():
            g2 = g.reshape(-1, g.shape[-1])
            res["dw"], res["db"] = _wgrad_and_bias(weight, ctx.bias_p, g2, total.reshape(-1, total.shape[-1]))
            _flush_wgrad()
        wt = _dgrad_weight_t(weight)
        gi = rs_ring(lambda lo, m, o: _dgrad_rows(g[lo:lo + m], weight, wt, o), group,
                     g.shape[:-1] + (weight.shape[1],), g, wgrad, bulk=ctx.bulk, defer_add=ctx.defer_add)
        if "dw" not in res:   # world 1 ring: no wait happened
            wgrad()
        return gi, res["dw"], res["db"], None


class _RowSPLinear(torch.autograd.Function):
    """Row-parallel linear whose output is reduce-scattered along the sequence: forward = per-chunk
    GEMMs fused with a ring reduce-scatter; backward = ring all-gather of the output gradient
    fused with the dgrad GEMM (queued weight gradients drained while the last chunk travels)."""

    @staticmethod
    def forward(ctx, x, weight):
        group = _tp_group()
        x = x.contiguous()
        ws = dist.get_world_size(group)
        assert x.shape[0] % ws == 0, "sequence length must divide the TP size"
        n = x.shape[0] // ws
        y = rs_ring(lambda lo, m, o: _linear_into(x[lo:lo + m], weight, o), group,
                    x.shape[:-1] + (weight.shape[0],), x)
        ctx.save_for_backward(x, weight)
        ctx.n = n
        ctx.bulk = _SPLIT["on"]
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight = ctx.saved_tensors
        group = _tp_group()
        g = g.contiguous()
        n = ctx.n
        gi = x.new_empty(x.shape)
        wt = _dgrad_weight_t(weight)
        gfull = ag_ring(g, group, lambda lo, ch: dgrad_into(gi[lo:lo + ch.shape[0]], ch, weight, wt),
                        before_last_wait=_flush_wgrad, bulk=ctx.bulk)
        dw = _wgrad(weight, gfull.reshape(-1, gfull.shape[-1]), x.reshape(-1, x.shape[-1]))
        return gi, dw


def _bias_grad(bias_p, g2):
    """Column sums of g2 into the bias' fp32 main_grad (returns None) or as a tensor."""
    if bias_p is None:
        return None
    tgt = SF.grad_accumulate_target(bias_p)
    if tgt is not None and g2.is_contiguous() and g2.shape[-1] % 8 == 0:
        _ext.ext().bias_grad(g2, tgt, True)
        bias_p._smdt_grad_ready(bias_p)
        return None
    return g2.sum(0)


def column_sp_linear(x, weight, bias):
    return _ColumnSPLinear.apply(x, weight, bias)


def row_sp_linear(x, weight):
    return _RowSPLinear.apply(x, weight)


# --------------------------------------------------------------------------------------------
# TP-invariant initialisation


def _key_seed(base_seed: int, key: str) -> int:
    h = hashlib.sha1(f"{base_seed}:{key}".encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 62) - 1)


_INIT = {"method": "normal", "perform": True, "cpu": False}


@contextlib.contextmanager
def weight_init(method: str = "normal", perform: bool = True, cpu: bool = False):
    """The init rule of the weights built inside (Megatron's ``--init-method-xavier-uniform`` /
    ``--no-initialization``, /root/reference/3_training_megatron-lm/megatron/arguments.py):
    ``"normal"`` draws N(0, std); ``"xavier_uniform"`` draws U(-a, a), a = sqrt(6 / (fan_in +
    fan_out)) of the FULL 2-D weight (so the values do not depend on the TP degree), for every
    weight, the scaled output layers included; ``perform=False`` leaves weights unset (they are
    about to be loaded from a checkpoint) and skips the full-tensor draw; ``cpu=True``
    (``--use-cpu-initialization``) draws on the host generator and moves the shard to the device,
    so a GPU model starts from exactly the CPU model's weights."""
    assert method in ("normal", "xavier_uniform"), method
    old = dict(_INIT)
    _INIT.update(method=method, perform=bool(perform), cpu=bool(cpu))
    try:
        yield
    finally:
        _INIT.update(old)


@torch.no_grad()
def init_full_then_shard(shape, std: float, key: str, base_seed: int, dtype, device, shard_dim: Optional[int],
                         rank: int, world: int, chunks=None):
    """Normal(0, std) init of the FULL tensor from a deterministic generator, then return this
    rank's shard along ``shard_dim``. ``chunks`` (a list of sizes along shard_dim) shards each
    chunk separately (fused QKV / gate-up weights keep per-rank [q|k|v] groups). ``weight_init``
    switches the rule (Xavier-uniform, or no initialization)."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if not _INIT["perform"]:
        sh = list(shape)
        if shard_dim is not None and world > 1:
            sh[shard_dim] //= world
        return torch.empty(sh, dtype=dtype, device=dev)
    if _INIT["cpu"] and dev.type != "cpu":
        with weight_init(_INIT["method"], True, False):
            return init_full_then_shard(shape, std, key, base_seed, dtype, None, shard_dim, rank, world,
                                        chunks).to(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(_key_seed(base_seed, key))
    full = torch.empty(shape, dtype=torch.float32, device=dev)
    if std == 0:
        full.zero_()
    elif _INIT["method"] == "xavier_uniform" and len(shape) == 2:
        a = math.sqrt(6.0 / (shape[0] + shape[1]))
        full.uniform_(-a, a, generator=gen)
    else:
        full.normal_(0.0, std, generator=gen)
    if shard_dim is None or world == 1:
        return full.to(dtype)
    if chunks is None:
        return full.chunk(world, dim=shard_dim)[rank].contiguous().to(dtype)
    parts = torch.split(full, chunks, dim=shard_dim)
    return torch.cat([p.chunk(world, dim=shard_dim)[rank] for p in parts], dim=shard_dim).contiguous().to(dtype)


class ColumnParallelLinear(nn.Module):
    """Y = X A with A split along its output dim: rank holds A[:, rank-slice]."""

    def __init__(self, input_size, output_size, bias=True, gather_output=False, init_std=0.02, key="col",
                 seed=1234, params_dtype=torch.float32, device=None, sequence_parallel=False,
                 skip_bias_add=False, chunks=None, async_tensor_model_parallel_allreduce=True,
                 bias_grad_from_output=False):
        super().__init__()
        st = ps.get_state()
        self.tp, self.rank = st.tp, st.tp_rank
        assert output_size % self.tp == 0, f"{output_size} not divisible by TP {self.tp}"
        self.input_size, self.output_size = input_size, output_size
        self.out_local = output_size // self.tp
        self.gather_output = gather_output
        self.sequence_parallel = sequence_parallel and self.tp > 1
        self.skip_bias_add = skip_bias_add
        # skip_bias_add and the caller only ever adds the returned bias to the output (h + b, e.g.
        # the fused bias-GeLU): the bias gradient equals the column sums of this linear's output
        # gradient, so the linear produces it with its weight gradient (one pass over dY) and the
        # returned bias is detached
        self.bias_grad_from_output = bool(bias_grad_from_output and skip_bias_add and bias)
        self.async_ar = async_tensor_model_parallel_allreduce and self.tp > 1 and not self.sequence_parallel
        w = init_full_then_shard((output_size, input_size), init_std, key + ".weight", seed, params_dtype, device, 0,
                                 self.rank, self.tp, chunks)
        self.weight = nn.Parameter(w)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 0
        if bias:
            self.bias = nn.Parameter(torch.zeros(self.out_local, dtype=params_dtype, device=device))
            self.bias.tensor_model_parallel = True
            self.bias.partition_dim = 0
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        if not (self.async_ar or self.sequence_parallel):
            x = copy_to_tensor_model_parallel_region(x)
        if self.bias_grad_from_output:
            y = linear_with_grad_accumulation_and_async_allreduce(x, self.weight, self.bias, self.sequence_parallel,
                                                                  self.async_ar, add_bias=False)
        else:
            b = None if self.skip_bias_add else self.bias
            y = linear_with_grad_accumulation_and_async_allreduce(x, self.weight, b, self.sequence_parallel,
                                                                  self.async_ar)
        if self.gather_output:
            y = gather_from_tensor_model_parallel_region(y)
        if self.skip_bias_add:
            return y, (self.bias.detach() if self.bias_grad_from_output else self.bias)
        return y


class RowParallelLinear(nn.Module):
    """Y = X A with A split along its input dim; partial outputs are all-reduced (or
    reduce-scattered along the sequence with sequence parallelism)."""

    def __init__(self, input_size, output_size, bias=True, input_is_parallel=True, init_std=0.02, key="row",
                 seed=1234, params_dtype=torch.float32, device=None, sequence_parallel=False,
                 skip_bias_add=False):
        super().__init__()
        st = ps.get_state()
        self.tp, self.rank = st.tp, st.tp_rank
        assert input_size % self.tp == 0
        self.input_size, self.output_size = input_size, output_size
        self.in_local = input_size // self.tp
        self.input_is_parallel = input_is_parallel
        self.sequence_parallel = sequence_parallel and self.tp > 1
        self.skip_bias_add = skip_bias_add
        w = init_full_then_shard((output_size, input_size), init_std, key + ".weight", seed, params_dtype, device, 1,
                                 self.rank, self.tp)
        self.weight = nn.Parameter(w)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 1
        if bias:
            self.bias = nn.Parameter(torch.zeros(output_size, dtype=params_dtype, device=device))
            self.bias.sequence_parallel = self.sequence_parallel
        else:
            self.register_parameter("bias", None)

    def forward(self, x):
        if not self.input_is_parallel:
            x = scatter_to_tensor_model_parallel_region(x)
        if self.sequence_parallel and _TP_OVERLAP:
            y = _RowSPLinear.apply(x, self.weight)
        elif self.sequence_parallel:
            y = linear_with_grad_accumulation_and_async_allreduce(x, self.weight, None, False, False)
            y = reduce_scatter_to_sequence_parallel_region(y)
        else:
            y = linear_with_grad_accumulation_and_async_allreduce(x, self.weight, None, False, False)
            y = reduce_from_tensor_model_parallel_region(y)
        if self.skip_bias_add:
            return y, self.bias
        return y + self.bias if self.bias is not None else y


class _EmbeddingLookup(torch.autograd.Function):
    """out = weight[ids]. Backward scatters the rows with ``index_add_`` (device atomics, no host
    synchronisation — torch's sort-based embedding backward stalls the CPU on the GPU and leaves
    the tail of every backward launch-bound), straight into the fp32 DDP ``main_grad`` when the
    weight has one (K7-style fusion: no dense bf16 [V, H] gradient, no cast pass)."""

    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.weight = weight
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        w = ctx.weight
        flat = ids.reshape(-1)
        g2 = g.reshape(-1, g.shape[-1]).float()
        mg = getattr(w, "main_grad", None)
        if mg is not None and mg.dtype == torch.float32:
            mg.index_add_(0, flat, g2)
            cb = getattr(w, "_smdt_grad_ready", None)
            if cb is not None:
                cb(w)
            return None, None
        dw = torch.zeros(w.shape, dtype=torch.float32, device=g.device)
        dw.index_add_(0, flat, g2)
        return None, dw.to(w.dtype)


class _AddPositionSlice(torch.autograd.Function):
    """e [s, b, h] + weight[start:start + s] broadcast over b. Backward: de = g, and the table's
    gradient is the batch sum of g (one reduction) added to rows start..start + s of the fp32
    ``main_grad`` (torch's embedding backward would scatter s * b rows with atomics)."""

    @staticmethod
    def forward(ctx, e, weight, start):
        s = e.shape[0]
        ctx.weight, ctx.start = weight, start
        return e + weight[start:start + s].unsqueeze(1)

    @staticmethod
    def backward(ctx, g):
        w, start = ctx.weight, ctx.start
        s = g.shape[0]
        gs = g.sum(1, dtype=torch.float32)                          # [s, h]
        mg = getattr(w, "main_grad", None)
        if mg is not None and mg.dtype == torch.float32:
            mg[start:start + s].add_(gs)
            cb = getattr(w, "_smdt_grad_ready", None)
            if cb is not None:
                cb(w)
            return g, None, None
        dw = torch.zeros(w.shape, dtype=torch.float32, device=g.device)
        dw[start:start + s] = gs
        return g, dw.to(w.dtype), None


def add_position_slice(e, weight, start: int):
    """e + weight[start:start + e.shape[0]] (learned absolute positions shared by every sequence)."""
    assert start + e.shape[0] <= weight.shape[0], "sequence longer than the position table"
    if not torch.is_grad_enabled() or not weight.requires_grad:
        return e + weight[start:start + e.shape[0]].unsqueeze(1)
    return _AddPositionSlice.apply(e, weight, int(start))


def embedding_lookup(ids, weight):
    """weight[ids] with the synchronisation-free backward above (torch's own path when
    deterministic algorithms are requested: atomics make the fp32 sum order run-dependent)."""
    if torch.are_deterministic_algorithms_enabled() or not torch.is_grad_enabled() or not weight.requires_grad:
        return F.embedding(ids, weight)
    return _EmbeddingLookup.apply(ids, weight)


class VocabParallelEmbedding(nn.Module):
    """Embedding table split along the vocab dim; out-of-range rows contribute zeros and the
    partial lookups are summed across TP (all-reduce, or reduce-scatter with SP)."""

    def __init__(self, num_embeddings, embedding_dim, init_std=0.02, key="embedding", seed=1234,
                 params_dtype=torch.float32, device=None):
        super().__init__()
        st = ps.get_state()
        self.tp, self.rank = st.tp, st.tp_rank
        assert num_embeddings % self.tp == 0, "pad the vocab to a multiple of TP (make-vocab-size-divisible-by)"
        self.num_embeddings = num_embeddings
        self.per = num_embeddings // self.tp
        self.vocab_start = self.rank * self.per
        self.vocab_end = self.vocab_start + self.per
        w = init_full_then_shard((num_embeddings, embedding_dim), init_std, key + ".weight", seed, params_dtype,
                                 device, 0, self.rank, self.tp)
        self.weight = nn.Parameter(w)
        self.weight.tensor_model_parallel = True
        self.weight.partition_dim = 0

    def forward(self, ids, reduce=True):
        if self.tp > 1:
            mask = (ids < self.vocab_start) | (ids >= self.vocab_end)
            local = (ids - self.vocab_start).masked_fill(mask, 0)
            out = embedding_lookup(local, self.weight)
            out = out.masked_fill(mask.unsqueeze(-1), 0.0)
            if reduce:
                out = reduce_from_tensor_model_parallel_region(out)
            return out
        return embedding_lookup(ids, self.weight)


# --------------------------------------------------------------------------------------------
# data broadcast within TP (U4)


def broadcast_data(keys, data, datatype, src_rank=None):
    """Broadcast {key: int tensor} from TP rank 0 to the TP group (sizes first, then a flat
    buffer), like Megatron's ``tensor_parallel.broadcast_data`` (`pretrain_gpt.py:75`)."""
    st = ps.get_state()
    if st.tp == 1 or st.tp_group is None:
        return {k: data[k].to(datatype) for k in keys}
    src = st.tp_ranks[0] if src_rank is None else src_rank
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if st.tp_rank == 0:
        sizes = []
        for k in keys:
            s = list(data[k].shape)
            sizes.append(len(s))
            sizes += s
        sz = torch.tensor(sizes + [0] * (32 * len(keys) - len(sizes)), dtype=torch.long, device=dev)
    else:
        sz = torch.zeros(32 * len(keys), dtype=torch.long, device=dev)
    dist.broadcast(sz, src, group=st.tp_group)
    shapes, i = [], 0
    szl = sz.tolist()
    for _ in keys:
        nd = szl[i]
        shapes.append(szl[i + 1:i + 1 + nd])
        i += 1 + nd
    total = sum(math.prod(s) for s in shapes)
    if st.tp_rank == 0:
        flat = torch.cat([data[k].to(dev).contiguous().view(-1).to(datatype) for k in keys])
    else:
        flat = torch.empty(total, dtype=datatype, device=dev)
    dist.broadcast(flat, src, group=st.tp_group)
    out, off = {}, 0
    for k, s in zip(keys, shapes):
        n = math.prod(s)
        out[k] = flat[off:off + n].view(s)
        off += n
    return out
