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

from ..parallel import state as ps


def _ddp_list(models):
    return [m for m in models if hasattr(m, "no_sync")]


class _SyncGate:
    """Enable DDP bucket launches only for the final backward pass of an iteration."""

    def __init__(self, models):
        self.ddps = _ddp_list(models)

    def set(self, enabled: bool):
        for d in self.ddps:
            d.sync_enabled = enabled


def forward_backward_no_pipelining(forward_step_func: Callable, data_iterator, model, num_microbatches: int,
                                   forward_only: bool = False, **_):
    """Gradient accumulation over ``num_microbatches``; returns the list of loss dicts.

    ``forward_step_func(data_iterator, model) -> (output_tensor, loss_func)`` with
    ``loss_func(output_tensor) -> (loss, {name: reduced})`` (Megatron's contract,
    `pretrain_gpt.py:92-117`).
    """
    models = model if isinstance(model, list) else [model]
    m = models[0]
    gate = _SyncGate(models)
    losses = []
    for i in range(num_microbatches):
        last = i == num_microbatches - 1
        gate.set(last)
        out, loss_func = forward_step_func(data_iterator, m)
        loss, info = loss_func(out)
        losses.append(info)
        if not forward_only:
            (loss / num_microbatches).backward()
    gate.set(True)
    return losses


# ------------------------------------------------------------------------------------ p2p


def _p2p(send_next=None, send_prev=None, recv_next_shape=None, recv_prev_shape=None, dtype=None, device=None):
    st = ps.get_state()
    ops = []
    rp = rn = None
    if send_prev is not None:
        ops.append(dist.P2POp(dist.isend, send_prev.contiguous(), st.prev_pp_rank))
    if recv_prev_shape is not None:
        rp = torch.empty(recv_prev_shape, dtype=dtype, device=device, requires_grad=True)
        ops.append(dist.P2POp(dist.irecv, rp, st.prev_pp_rank))
    if send_next is not None:
        ops.append(dist.P2POp(dist.isend, send_next.contiguous(), st.next_pp_rank))
    if recv_next_shape is not None:
        rn = torch.empty(recv_next_shape, dtype=dtype, device=device, requires_grad=True)
        ops.append(dist.P2POp(dist.irecv, rn, st.next_pp_rank))
    if ops:
        for r in dist.batch_isend_irecv(ops):
            r.wait()
    return rp, rn


def forward_backward_pipelining_without_interleaving(forward_step_func: Callable, data_iterator, model,
                                                     num_microbatches: int, tensor_shape, dtype=torch.bfloat16,
                                                     forward_only: bool = False, **_):
    """1F1B. ``tensor_shape`` is the [s(/tp), b, h] activation exchanged between stages."""
    models = model if isinstance(model, list) else [model]
    m = models[0]
    st = ps.get_state()
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    first, last = st.is_first_stage(), st.is_last_stage()
    gate = _SyncGate(models)
    gate.set(False)
    warm = min(st.pp - st.pp_rank - 1, num_microbatches)
    steady = num_microbatches - warm
    inputs: List[Optional[torch.Tensor]] = []
    outputs: List[torch.Tensor] = []
    losses = []
    n_backward = [0]

    def fwd(inp):
        core = m.module if hasattr(m, "module") else m
        core.set_input_tensor(inp)
        out, loss_func = forward_step_func(data_iterator, m)
        if last:
            loss, info = loss_func(out)
            losses.append(info)
            return loss / num_microbatches
        return out

    def bwd(inp, out, gout):
        n_backward[0] += 1
        gate.set(n_backward[0] == num_microbatches)
        if inp is not None:
            inp.retain_grad()
        if gout is None:
            torch.autograd.backward(out)
        else:
            torch.autograd.backward(out, grad_tensors=gout)
        return None if inp is None else inp.grad

    def recv_fwd():
        return None if first else _p2p(recv_prev_shape=tensor_shape, dtype=dtype, device=dev)[0]

    def recv_bwd():
        return None if last else _p2p(recv_next_shape=tensor_shape, dtype=dtype, device=dev)[1]

    for _ in range(warm):
        inp = recv_fwd()
        out = fwd(inp)
        if not last:
            _p2p(send_next=out)
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
        inputs.append(inp)
        outputs.append(out)
        i0, o0 = inputs.pop(0), outputs.pop(0)
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
    if not forward_only:
        for _ in range(warm):
            i0, o0 = inputs.pop(0), outputs.pop(0)
            gout = recv_bwd()
            gin = bwd(i0, o0, gout)
            if not first:
                _p2p(send_prev=gin)
    gate.set(True)
    return losses


def get_forward_backward_func():
    st = ps.get_state()
    if st.pp > 1:
        return forward_backward_pipelining_without_interleaving
    return forward_backward_no_pipelining
