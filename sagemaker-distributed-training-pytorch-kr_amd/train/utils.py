"""Training utilities with Megatron semantics.

``get_ltor_masks_and_position_ids`` (`pretrain_gpt.py:83-88`) and
``average_losses_across_data_parallel_group`` (`pretrain_gpt.py:98`) from the reference recipe.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..parallel import state as ps


def get_ltor_masks_and_position_ids(data, eod_token, reset_position_ids=False, reset_attention_mask=False,
                                    eod_mask_loss=False, build_attention_mask=True):
    """Left-to-right masks. Returns (attention_mask [b or 1, 1, s, s] bool True=masked | None,
    loss_mask [b, s] float, position_ids [b, s] long).

    With flash attention the causal mask is implicit, so the dense mask is only materialised
    when ``reset_attention_mask`` needs per-document blocks or ``build_attention_mask`` asks.
    """
    b, s = data.shape
    att_b = b if reset_attention_mask else 1
    attention_mask = None
    if build_attention_mask or reset_attention_mask:
        attention_mask = torch.tril(torch.ones((att_b, s, s), device=data.device)).view(att_b, 1, s, s)
    loss_mask = torch.ones(data.shape, dtype=torch.float, device=data.device)
    if eod_mask_loss:
        loss_mask[data == eod_token] = 0.0
    position_ids = torch.arange(s, dtype=torch.long, device=data.device).unsqueeze(0).expand_as(data)
    if reset_position_ids:
        position_ids = position_ids.clone()
    if reset_position_ids or reset_attention_mask:
        for bi in range(b):
            eod_idx = (data[bi] == eod_token).nonzero().view(-1).tolist()
            prev = 0
            for j in eod_idx:
                if reset_attention_mask:
                    attention_mask[bi, 0, (j + 1):, :(j + 1)] = 0
                if reset_position_ids:
                    position_ids[bi, (j + 1):] -= (j + 1 - prev)
                    prev = j + 1
    if attention_mask is not None:
        attention_mask = attention_mask < 0.5
    if not reset_position_ids:
        # plain 0 .. s-1 in every row: lets GPTModel add the position table as a broadcast slice
        # (a tensor derived from this one by slicing / copying loses the mark and takes the gather)
        position_ids._smdt_arange_start = 0
    return attention_mask, loss_mask, position_ids


def average_losses_across_data_parallel_group(losses):
    """All-reduce scalars over DP (x CP: context-parallel ranks hold different tokens of the same
    samples) and divide by the group size (once per micro-batch)."""
    avg = torch.cat([l.clone().detach().view(1).float() for l in losses])
    st = ps.get_state()
    group = st.dp_cp_group if getattr(st, "cp", 1) > 1 else st.dp_group
    n = st.dp * getattr(st, "cp", 1)
    if dist.is_initialized() and n > 1 and group is not None:
        dist.all_reduce(avg, group=group)
        avg = avg / n
    return avg


def context_parallel_slice(*tensors, dim: int = 1):
    """This context-parallel rank's contiguous sequence chunk of each [b, s, ...] batch tensor
    (tokens, labels, loss mask, position ids); identity when cp = 1."""
    st = ps.get_state()
    cp = getattr(st, "cp", 1)
    if cp == 1:
        return tensors if len(tensors) != 1 else tensors[0]
    out = []
    for t in tensors:
        if t is None:
            out.append(None)
            continue
        assert t.shape[dim] % cp == 0, f"sequence {t.shape[dim]} not divisible by context-parallel size {cp}"
        out.append(t.chunk(cp, dim=dim)[st.cp_rank].contiguous())
    return tuple(out) if len(out) != 1 else out[0]


def report_memory(name: str) -> str:
    mb = 1024.0 * 1024.0
    if not torch.cuda.is_available():
        return f"[Rank {dist.get_rank() if dist.is_initialized() else 0}] ({name}) memory (MB) | n/a (cpu)"
    s = (f"[Rank {dist.get_rank() if dist.is_initialized() else 0}] ({name}) memory (MB)"
         f" | allocated: {torch.cuda.memory_allocated() / mb}"
         f" | max allocated: {torch.cuda.max_memory_allocated() / mb}"
         f" | reserved: {torch.cuda.memory_reserved() / mb}"
         f" | max reserved: {torch.cuda.max_memory_reserved() / mb}")
    return s


def unwrap_model(model):
    while hasattr(model, "module"):
        model = model.module
    return model
