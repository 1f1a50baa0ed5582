"""Forward/backward schedules: no pipelining (gradient accumulation) and pipeline-parallel
1F1B (non-interleaved and interleaved virtual stages), with p2p over RCCL/xGMI.

Megatron equivalents: ``forward_backward_no_pipelining`` and
``forward_backward_pipelining_without/with_interleaving``; flags `--pipeline-model-parallel-size`,
`--num-layers-per-virtual-pipeline-stage`, `--overlap-p2p-communication`
(/root/reference/3_training_megatron-lm/megatron/arguments.py:1004-1017).

Gradient all-reduce overlap: the DDP reducer is disabled for every micro-batch except the last
backward, so bucket collectives fire only once (during that final backward).
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from ..comm import stats as _cs
from ..parallel import state as ps
from .pipeline_sim import warmup_and_defer


def _ddp_list(models):
    return [m for m in models if hasattr(m, "no_sync")]


class _SyncGate:
    """Enable DDP bucket launches only for the final backward pass of an iteration."""

    def __init__(self, models):
        self.ddps = _ddp_list(models)

    def set(self, enabled: bool):
        for d in self.ddps:
            if hasattr(d, "set_sync_enabled"):
                d.set_sync_enabled(enabled)
            else:
                d.sync_enabled = enabled


def _scaled(loss, num_microbatches, grad_scale):
    """Megatron's ``optimizer.scale_loss``: 1 / num_microbatches and the fp16 loss scale (a device
    tensor — no host sync) applied to the loss before backward."""
    loss = loss / num_microbatches
    return loss * grad_scale if grad_scale is not None else loss


def forward_backward_no_pipelining(forward_step_func: Callable, data_iterator, model, num_microbatches: int,
                                   forward_only: bool = False, grad_scale=None, split_backward: bool = False, **_):
    """Gradient accumulation over ``num_microbatches``; returns the list of loss dicts.

    ``forward_step_func(data_iterator, model) -> (output_tensor, loss_func)`` with
    ``loss_func(output_tensor) -> (loss, {name: reduced})`` (Megatron's contract,
    `pretrain_gpt.py:92-117`).

    ``split_backward``: each micro-batch's weight-gradient GEMMs are held for the whole backward
    (``DEFERRED_WGRAD.defer``) and issued as one grouped launch after it — the W work of one
    micro-batch exactly as a stage of the zero-bubble pipeline schedules issues it. bench.py's
    per-rank emulation of a pipeline stage (``--emulate-tp``) runs this way, so the measured
    stage time has the schedule's W grouping instead of the opportunistic per-collective flushes
    of a plain backward.
    """
    from ..parallel.tensor_parallel import DEFERRED_WGRAD, W_FILL, accumulation_window_ok, forward_fill
    models = model if isinstance(model, list) else [model]
    m = models[0]
    gate = _SyncGate(models)
    # SMDT_W_FILL: a micro-batch's W stays queued into the next forward, whose TP-exchange waits
    # issue it piece by piece (parallel/tensor_parallel.fill_exchange_wait)
    fill = split_backward and W_FILL and not forward_only
    # opt-in (SMDT_WGRAD_MERGE_ACCUM=1): the micro-batches' weight-gradient GEMMs merge per weight
    # and run once, in the last backward (DeferredWgrad.hold): one fp32 main_grad update per
    # iteration; it loses at Megatron's usual micro-batch sizes (profiles/r3_l4l/)
    hold = not forward_only and num_microbatches > 1 and accumulation_window_ok(gate.ddps, default=False)
    losses = []
    for i in range(num_microbatches):
        last = i == num_microbatches - 1
        gate.set(last)                   # (re-enabling sync does not drain a held window)
        if hold:
            DEFERRED_WGRAD.hold = not last
        if fill:
            with forward_fill():
                out, loss_func = forward_step_func(data_iterator, m)
        else:
            out, loss_func = forward_step_func(data_iterator, m)
        loss, info = loss_func(out)
        losses.append(info)
        if not forward_only:
            if split_backward:
                DEFERRED_WGRAD.defer = True
            try:
                if fill:
                    with forward_fill(flush_end=False):   # B's exchange waits take queued W too
                        _scaled(loss, num_microbatches, grad_scale).backward()
                else:
                    _scaled(loss, num_microbatches, grad_scale).backward()
            finally:
                if split_backward:
                    DEFERRED_WGRAD.defer = False
            if split_backward and (last or not fill):
                DEFERRED_WGRAD.flush()
    gate.set(True)
    return losses


# ------------------------------------------------------------------------------------ p2p


class P2PConfig:
    """Pipeline p2p behaviour (Megatron flags, /root/reference/3_training_megatron-lm/megatron/
    arguments.py:1014-1037):

    * ``overlap`` (--overlap-p2p-communication): receives are not waited for where they are
      issued but right before their consumer (the next forward / backward), so the RCCL transfer
      runs beside the compute issued in between (on ROCm a wait is a stream dependency, not a
      host block, so deferring it is what lets the MFMA work start).
    * ``scatter_gather`` (default on; --no-scatter-gather-tensors-in-pipeline turns it off): with
      TP > 1 and no sequence parallelism each TP rank sends only its 1/tp slice of the (TP-
      replicated) activation and the receiver all-gathers it over TP — tp x fewer p2p bytes.
    * ``deallocate_outputs`` (Megatron's deallocate_pipeline_outputs): once an activation was sent
      to the next stage its data is dropped (only its autograd graph is needed), and backward
      runs through the autograd engine directly.

    Send-only groups are never waited for where they are issued; every in-flight send is
    retired at the end of the schedule.
    """

    def __init__(self, overlap=False, scatter_gather=True, deallocate_outputs=True):
        self.overlap = overlap
        self.scatter_gather = scatter_gather
        self.deallocate_outputs = deallocate_outputs


_P2P = P2PConfig()
_INFLIGHT_SENDS: List = []


def configure_p2p(args=None, **kw):
    """Set the pipeline p2p behaviour from parsed Megatron args (or keywords)."""
    global _P2P
    if args is not None:
        if getattr(args, "use_ring_exchange_p2p", False):
            raise ValueError("--use-ring-exchange-p2p needs torch.distributed.ring_exchange (a patched PyTorch "
                             "build); on ROCm use the default batched RCCL p2p")
        kw.setdefault("overlap", bool(getattr(args, "overlap_p2p_communication", False)))
        kw.setdefault("scatter_gather", bool(getattr(args, "scatter_gather_tensors_in_pipeline", True)))
        kw.setdefault("deallocate_outputs", bool(getattr(args, "deallocate_pipeline_outputs", True)))
    _P2P = P2PConfig(**kw)
    return _P2P


def get_p2p_config():
    return _P2P


_SCHED = {"sp": False}


def _enter_schedule(model):
    """Per-schedule p2p context: scatter-gather applies only to TP-replicated activations (no
    sequence parallelism — SP activations are already TP-sharded)."""
    m = model[0] if isinstance(model, (list, tuple)) else model
    core = m.module if hasattr(m, "module") else m
    if isinstance(core, torch.nn.ModuleList) and len(core):
        core = core[0]
    cfg = getattr(core, "cfg", None)
    _SCHED["sp"] = bool(getattr(cfg, "sequence_parallel", False))


def _sg_active():
    st = ps.get_state()
    return _P2P.scatter_gather and st.tp > 1 and st.tp_group is not None and not _SCHED["sp"]


def _sg_slice(t):
    st = ps.get_state()
    return t.contiguous().view(-1).chunk(st.tp)[st.tp_rank].contiguous()


def _finish_recv(t):
    """Wait for a received tensor's transfer (deferred under ``overlap``) and, with scatter-gather,
    all-gather its TP slices back into the full activation. Returns the usable tensor."""
    if t is None:
        return None
    holder = getattr(t, "_smdt_works", None)
    if holder is not None and holder[0] is not None:
        # one p2p group may carry both receives: its works are waited exactly once (a second
        # wait on a retired gloo send blocks for a send that never comes)
        works, holder[0] = holder[0], None
        with _cs.waiting("pp"):
            for w in works:
                w.wait()
    t._smdt_works = None
    full_shape = getattr(t, "_smdt_sg_shape", None)
    if full_shape is not None:
        st = ps.get_state()
        full = torch.empty((t.numel() * st.tp,), dtype=t.dtype, device=t.device)
        with _cs.blocking("all_gather", st.tp_group, full.numel() * full.element_size()):
            dist.all_gather_into_tensor(full, t.detach(), group=st.tp_group)
        out = full.view(full_shape).requires_grad_(True)
        t._smdt_sg_shape = None
        t._smdt_full = out
        return out
    full = getattr(t, "_smdt_full", None)
    return t if full is None else full


def _p2p(send_next=None, send_prev=None, recv_next_shape=None, recv_prev_shape=None, dtype=None, device=None):
    st = ps.get_state()
    ops = []
    rp = rn = None
    sg = _sg_active()

    def _recv_buf(shape):
        if sg:
            n = 1
            for d in shape:
                n *= d
            t = torch.empty((n // st.tp,), dtype=dtype, device=device)
            t._smdt_sg_shape = tuple(shape)
            return t
        return torch.empty(shape, dtype=dtype, device=device, requires_grad=True)

    def _send_buf(t):
        # a detached alias: dropping the activation's data after the send cannot free the storage
        # the transfer still reads (the work keeps the alias alive)
        return _sg_slice(t.detach()) if sg else t.detach().contiguous()
    # Canonical order — activations (to next / from prev) before gradients (to prev / from next)
    # on every rank — so the per-peer message streams match even when next == prev (a 2-rank
    # ring in the interleaved schedule): RCCL pairs point-to-point ops per peer in issue order.
    if send_next is not None:
        ops.append(dist.P2POp(dist.isend, _send_buf(send_next), st.next_pp_rank))
    if recv_prev_shape is not None:
        rp = _recv_buf(recv_prev_shape)
        ops.append(dist.P2POp(dist.irecv, rp, st.prev_pp_rank))
    if send_prev is not None:
        ops.append(dist.P2POp(dist.isend, _send_buf(send_prev), st.prev_pp_rank))
    if recv_next_shape is not None:
        rn = _recv_buf(recv_next_shape)
        ops.append(dist.P2POp(dist.irecv, rn, st.next_pp_rank))
    if not ops:
        return rp, rn
    works = dist.batch_isend_irecv(ops)
    if _cs._ON:
        sent = sum(o.tensor.numel() * o.tensor.element_size() for o in ops if o.op is dist.isend)
        _cs.collective("p2p", st.pp_group, sent, work=works[0] if len(works) == 1 else None)
    if rp is None and rn is None:
        _INFLIGHT_SENDS.extend(works)        # send-only: retired at the end of the schedule
        return rp, rn
    holder = [works]
    for t in (rp, rn):
        if t is not None:
            t._smdt_works = holder
    if not _P2P.overlap:
        rp, rn = _finish_recv(rp), _finish_recv(rn)
    return rp, rn


def _retire_sends():
    with _cs.waiting("pp"):
        while _INFLIGHT_SENDS:
            _INFLIGHT_SENDS.pop().wait()


def _drop_output(out):
    """Megatron's deallocate_output_tensor: after ``out`` went to the next stage only its graph
    is needed; its [s, b, h] data is replaced by one element."""
    if _P2P.deallocate_outputs and out is not None and out.grad_fn is not None and out._base is None:
        out.data = torch.empty((1,), device=out.device, dtype=out.dtype)


def _run_backward(out, gout):
    if gout is None:
        torch.autograd.backward(out)
    elif out.numel() != gout.numel():    # data was dropped after the send: call the engine directly
        torch.autograd.Variable._execution_engine.run_backward(
            tensors=(out,), grad_tensors=(gout,), keep_graph=False, create_graph=False, inputs=(),
            allow_unreachable=True, accumulate_grad=True)
    else:
        torch.autograd.backward(out, grad_tensors=gout)


# Non-interleaved pipeline schedule (``--pp-schedule``; train/pipeline_sim.py simulates each):
#   1f1b : Megatron's 1F1B — a stage's weight-gradient GEMMs run inside its backward pass, before
#          the input gradient is sent to the previous stage;
#   zb   : the backward split zero-bubble style: B (the input-gradient chain) runs with the
#          deferred wgrad queue held, the input gradient is SENT, then the stage's W GEMMs run
#          while it travels — the previous stage waits for B only;
#   zbh1 : zb, and rank r also keeps the W of its last r + 1 backward passes queued behind its
#          last B (ZB-H1): the final B chain the earlier stages wait for in the cooldown is not
#          held up by W work, which then fills their drain instead. Same activation memory as
#          1F1B; the held W operands (dY, X) of up to pp micro-batches stay in HBM.
#   zbh2 : ZB-H2-style: rank r runs 2 (pp - r - 1) forwards ahead and defers the W of its last
#          2 (r + 1) passes. Up to 2 (pp - r) - 1 micro-batches of activations in flight on stage
#          r — HBM the 288 GB part has to spare — for a bubble of just the last stage's first wait
#          (train/pipeline_sim.py: 16.2 -> 9.6 ms at the tp2pp2 BASELINE point).
PP_SCHEDULES = ("1f1b", "zb", "zbh1", "zbh2")
# library default: Megatron's 1F1B (the reference's schedule, no extra held W operands); the
# zero-bubble forms are opt-in (``--pp-schedule`` here and in bench.py, which selects zbh2)
_PP_SCHEDULE = {"name": "1f1b"}


def set_pipeline_schedule(name: str):
    if name not in PP_SCHEDULES:
        raise ValueError(f"--pp-schedule must be one of {PP_SCHEDULES}, got {name!r}")
    _PP_SCHEDULE["name"] = name


def get_pipeline_schedule() -> str:
    return _PP_SCHEDULE["name"]


def forward_backward_pipelining_without_interleaving(forward_step_func: Callable, data_iterator, model,
                                                     num_microbatches: int, tensor_shape, dtype=torch.bfloat16,
                                                     forward_only: bool = False, grad_scale=None, schedule=None, **_):
    """1F1B, optionally with the split (zero-bubble) backward of ``set_pipeline_schedule``.
    ``tensor_shape`` is the [s(/tp), b, h] activation exchanged between stages."""
    from ..parallel.tensor_parallel import DEFERRED_WGRAD, W_FILL, forward_fill
    models = model if isinstance(model, list) else [model]
    m = models[0]
    _enter_schedule(m)
    st = ps.get_state()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    first, last = st.is_first_stage(), st.is_last_stage()
    gate = _SyncGate(models)
    gate.set(False)
    schedule = schedule or get_pipeline_schedule()
    warm, defer_from = warmup_and_defer(schedule if not forward_only else "1f1b", st.pp, st.pp_rank,
                                        num_microbatches)
    steady = num_microbatches - warm
    inputs: List[Optional[torch.Tensor]] = []
    outputs: List[torch.Tensor] = []
    losses = []
    n_backward = [0]
    split = schedule in ("zb", "zbh1", "zbh2") and not forward_only and DEFERRED_WGRAD.enabled
    # zbh1 / zbh2: backward passes >= defer_from keep their W queued until after the last B
    concat0 = DEFERRED_WGRAD.concat_segments

    fill = split and W_FILL

    def fwd(inp):
        core = m.module if hasattr(m, "module") else m
        inp = _finish_recv(inp)
        core.set_input_tensor(inp)
        if fill:
            with forward_fill():     # the exchange waits issue the queued W of the last pass
                out, loss_func = forward_step_func(data_iterator, m)
        else:
            out, loss_func = forward_step_func(data_iterator, m)
        if last:
            loss, info = loss_func(out)
            losses.append(info)
            return _scaled(loss, num_microbatches, grad_scale)
        return out

    def bwd(inp, out, gout):
        k = n_backward[0]
        n_backward[0] += 1
        sync = n_backward[0] == num_microbatches
        if split:
            # queued W items of this pass: held (merged with the sync pass's, no readiness of their
            # own) when they stay queued beyond it; enabling sync must not flush earlier held ones
            held = k >= defer_from and not sync
            DEFERRED_WGRAD.defer = True
            DEFERRED_WGRAD.hold = held or (sync and k > defer_from)
            gate.set(sync)
            DEFERRED_WGRAD.hold = held
        else:
            gate.set(sync)
        inp, gout = _finish_recv(inp), _finish_recv(gout)
        if inp is not None:
            inp.retain_grad()
        if fill:
            with forward_fill(flush_end=False):   # B's exchange waits take queued W too
                _run_backward(out, gout)
        else:
            _run_backward(out, gout)
        if split:
            DEFERRED_WGRAD.defer = False
        return None if inp is None else inp.grad

    def after_send(k, forward_follows=False):
        """W of backward pass k, once its input gradient is on its way (split schedules). With
        SMDT_W_FILL and a forward next, it stays queued for that forward's exchange waits."""
        if split and (k < defer_from or k == num_microbatches - 1):
            DEFERRED_WGRAD.hold = False
            if not (fill and forward_follows):
                DEFERRED_WGRAD.flush()

    def recv_fwd():
        return None if first else _p2p(recv_prev_shape=tensor_shape, dtype=dtype, device=dev)[0]

    def recv_bwd():
        return None if last else _p2p(recv_next_shape=tensor_shape, dtype=dtype, device=dev)[1]

    if split:
        DEFERRED_WGRAD.concat_segments = False     # held + sync segments: one launch per round
    try:
        for _ in range(warm):
            inp = recv_fwd()
            out = fwd(inp)
            if not last:
                _p2p(send_next=out)
                _drop_output(out)
            inputs.append(inp)
            outputs.append(out)
        inp = recv_fwd() if steady > 0 else None
        for i in range(steady):
            is_last_iter = i == steady - 1
            out = fwd(inp)
            if forward_only:
                if not last:
                    _p2p(send_next=out)
                if not is_last_iter:
                    inp = recv_fwd()
                continue
            if last:
                gout = None
            else:
                gout = _p2p(send_next=out, recv_next_shape=tensor_shape, dtype=dtype, device=dev)[1]
                _drop_output(out)
            inputs.append(inp)
            outputs.append(out)
            i0, o0 = inputs.pop(0), outputs.pop(0)
            k = n_backward[0]
            gin = bwd(i0, o0, gout)
            if is_last_iter:
                inp = None
                if not first:
                    _p2p(send_prev=gin)
            else:
                if first:
                    inp = None
                    inp = recv_fwd()
                else:
                    inp = _p2p(send_prev=gin, recv_prev_shape=tensor_shape, dtype=dtype, device=dev)[0]
            after_send(k, forward_follows=not is_last_iter)
        if not forward_only:
            for _ in range(warm):
                i0, o0 = inputs.pop(0), outputs.pop(0)
                gout = recv_bwd()
                k = n_backward[0]
                gin = bwd(i0, o0, gout)
                if not first:
                    _p2p(send_prev=gin)
                after_send(k)
    finally:
        if split:
            DEFERRED_WGRAD.defer = False
            DEFERRED_WGRAD.hold = False
            DEFERRED_WGRAD.concat_segments = concat0
    _retire_sends()
    gate.set(True)
    return losses


# ------------------------------------------------------------------- interleaved (virtual) 1F1B


def _chunks_of(model):
    core = model.module if hasattr(model, "module") else model
    if isinstance(core, torch.nn.ModuleList):
        return list(core), model
    if isinstance(model, list):
        return model, model
    return [core], model


def _p2p_pair(send_next=None, send_prev=None, recv_prev=False, recv_next=False, shape=None, dtype=None,
              device=None):
    rp, rn = _p2p(send_next=send_next, send_prev=send_prev, recv_prev_shape=shape if recv_prev else None,
                  recv_next_shape=shape if recv_next else None, dtype=dtype, device=device)
    return rp, rn


def forward_backward_pipelining_with_interleaving(forward_step_func: Callable, data_iterator, model,
                                                  num_microbatches: int, tensor_shape, dtype=torch.bfloat16,
                                                  forward_only: bool = False, grad_scale=None, **_):
    """Interleaved 1F1B over ``vpp`` model chunks per pipeline rank (Megatron's virtual pipeline,
    `--num-layers-per-virtual-pipeline-stage`). Chunk c of rank r holds global stage c * pp + r,
    so activations travel the rank ring pp times per micro-batch; the pipeline bubble shrinks
    by a factor vpp. ``data_iterator`` may be one iterator (tee'd per chunk) or a list.

    Micro-batch k (of vpp * num_microbatches forward/backward units) runs on chunk
    ``(k % (pp * vpp)) // pp`` (reversed for backward); warm-up depth on rank r is
    ``2 (pp - r - 1) + (vpp - 1) pp``.
    """
    import itertools

    chunks, ddp = _chunks_of(model)
    _enter_schedule(chunks[0])
    vpp = len(chunks)
    st = ps.get_state()
    pp, r = st.pp, st.pp_rank
    if num_microbatches % pp != 0:
        raise ValueError(f"interleaved schedule needs num_microbatches ({num_microbatches}) divisible by pp ({pp})")
    if not isinstance(data_iterator, (list, tuple)):
        data_iterator = list(itertools.tee(data_iterator, vpp)) if data_iterator is not None else [None] * vpp
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    gate = _SyncGate([ddp] if hasattr(ddp, "no_sync") else [])
    gate.set(False)
    total = num_microbatches * vpp
    all_warmup = False
    if forward_only:
        warm = total
    elif num_microbatches == pp:
        warm, all_warmup = total, True
    else:
        warm = min((pp - r - 1) * 2 + (vpp - 1) * pp, total)
    remaining = total - warm
    inputs = [[] for _ in range(vpp)]
    outputs = [[] for _ in range(vpp)]
    ograds = [[] for _ in range(vpp)]
    losses = []
    n_backward = [0]

    def chunk_id(k, forward):
        c = (k % (pp * vpp)) // pp
        return c if forward else vpp - c - 1

    def set_vr(c):
        st.virtual_pp_rank = c

    def fwd_step(k):
        c = chunk_id(k, True)
        set_vr(c)
        if st.is_first_stage() and len(inputs[c]) == len(outputs[c]):
            inputs[c].append(None)
        inp = inputs[c][-1] = _finish_recv(inputs[c][-1])
        chunks[c].set_input_tensor(inp)
        out, loss_func = forward_step_func(data_iterator[c], chunks[c])
        if st.is_last_stage():
            loss, info = loss_func(out)
            losses.append(info)
            out = _scaled(loss, num_microbatches, grad_scale)
        outputs[c].append(out)
        return out

    def bwd_step(k):
        c = chunk_id(k, False)
        set_vr(c)
        if st.is_last_stage() and len(ograds[c]) == 0:
            ograds[c].append(None)
        inp, out, gout = inputs[c].pop(0), outputs[c].pop(0), _finish_recv(ograds[c].pop(0))
        n_backward[0] += 1
        gate.set(n_backward[0] == total)
        if inp is not None:
            inp.retain_grad()
        _run_backward(out, gout)
        return None if inp is None else inp.grad

    kw = dict(shape=tensor_shape, dtype=dtype, device=dev)
    set_vr(0)
    if not st.is_first_stage(ignore_virtual=True):
        inputs[0].append(_p2p_pair(recv_prev=True, **kw)[0])
    for k in range(warm):
        out = fwd_step(k)
        nxt = chunk_id(k + 1, True)
        recv_prev = not (st.is_first_stage(ignore_virtual=True) and nxt == 0) and k != total - 1
        if st.is_last_stage():
            out = None
        if k == warm - 1 and not forward_only and not all_warmup:
            recv_next = not st.is_last_stage(ignore_virtual=True)
            rp, rn = _p2p_pair(send_next=out, recv_prev=recv_prev, recv_next=recv_next, **kw)
            _drop_output(out)
            ograds[vpp - 1].append(rn)
        else:
            rp, _ = _p2p_pair(send_next=out, recv_prev=recv_prev, **kw)
            _drop_output(out)
        if recv_prev:
            inputs[nxt].append(rp)
    for k in range(remaining):
        fk, bk = k + warm, k
        out = fwd_step(fk)
        gin = bwd_step(bk)
        set_vr(chunk_id(fk, True))
        if st.is_last_stage():
            out = None
        set_vr(chunk_id(bk, False))
        if st.is_first_stage():
            gin = None
        recv_prev = True
        if st.is_first_stage(ignore_virtual=True):
            nxt_f = chunk_id(fk - (pp - 1), True)
            if nxt_f == vpp - 1:
                recv_prev = False
            nxt_f += 1
        else:
            nxt_f = chunk_id(fk + 1, True)
        recv_next = True
        if st.is_last_stage(ignore_virtual=True):
            nxt_b = chunk_id(bk - (pp - 1), False)
            if nxt_b == 0:
                recv_next = False
            nxt_b -= 1
        else:
            nxt_b = chunk_id(bk + 1, False)
        if k == remaining - 1:
            recv_prev = False
        rp, rn = _p2p_pair(send_next=out, send_prev=gin, recv_prev=recv_prev, recv_next=recv_next, **kw)
        _drop_output(out)
        if recv_prev:
            inputs[nxt_f].append(rp)
        if recv_next:
            ograds[nxt_b].append(rn)
    if not forward_only:
        if all_warmup:
            set_vr(vpp - 1)
            ograds[vpp - 1].append(None if st.is_last_stage(ignore_virtual=True)
                                   else _p2p_pair(recv_next=True, **kw)[1])
        for k in range(remaining, total):
            gin = bwd_step(k)
            if st.is_first_stage():
                gin = None
            nxt_b = chunk_id(k + 1, False)
            recv_next = not (st.is_last_stage(ignore_virtual=True) and nxt_b == vpp - 1) and k != total - 1
            _, rn = _p2p_pair(send_prev=gin, recv_next=recv_next, **kw)
            if recv_next:
                ograds[nxt_b].append(rn)
    set_vr(0)
    _retire_sends()
    gate.set(True)
    return losses


def get_forward_backward_func():
    st = ps.get_state()
    if st.pp > 1:
        if st.virtual_pp is not None and st.virtual_pp > 1:
            return forward_backward_pipelining_with_interleaving
        return forward_backward_pipelining_without_interleaving
    return forward_backward_no_pipelining
