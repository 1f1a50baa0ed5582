"""Stream priority for communication.

The reference makes sequence parallelism and async tensor-parallel all-reduce depend on an
ordering guarantee: Megatron refuses SP unless CUDA_DEVICE_MAX_CONNECTIONS=1
(/root/reference/3_training_megatron-lm/megatron/arguments.py:347-355; set at
/root/reference/3_training_megatron-lm/pretrain_gpt.py:14), so a collective issued before a GEMM
is dispatched before it. On MI355X the risk is not issue order but dispatch: an exchange or relay
kernel with bounded spins queued behind a 256-CU chunk GEMM that owns every CU. HIP's stream
priority lets the dispatcher place a high-priority stream's workgroups first as CUs free up.

Every communication side stream of the framework (xGMI engine, relay, direct TP exchange, smddp,
ZeRO-3 parameter movement, the loopback stand-ins of rank emulation) comes from ``comm_stream``,
and RCCL process groups get ``is_high_priority_stream`` (``nccl_pg_options``).
``SMDT_COMM_PRIORITY=normal`` turns both off (A/B: profiles/r5_priority/).
"""
from __future__ import annotations

import os

import torch

_STATE = {"cache": {}}


def high_priority() -> bool:
    return os.environ.get("SMDT_COMM_PRIORITY", "high") != "normal"


def priority_value() -> int:
    """The stream priority communication streams use (torch: lower = more urgent)."""
    if not high_priority() or not torch.cuda.is_available():
        return 0
    lo, hi = torch.cuda.Stream.priority_range()       # (least, greatest) urgency, e.g. (0, -1)
    return int(hi)


def comm_stream(device=None) -> "torch.cuda.Stream":
    """A new side stream for communication work, at high priority unless SMDT_COMM_PRIORITY=normal."""
    return torch.cuda.Stream(device=device, priority=priority_value())


def nccl_pg_options():
    """``pg_options`` for RCCL groups: the communicator's internal stream at high priority
    (None when off, or when this torch has no ProcessGroupNCCL)."""
    if not high_priority():
        return None
    try:
        from torch.distributed import ProcessGroupNCCL
    except ImportError:
        return None
    opts = ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def describe() -> dict:
    return {"comm_stream_priority": "high" if high_priority() else "normal",
            "priority_value": priority_value()}
