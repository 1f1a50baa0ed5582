"""Process-group topology: tensor / pipeline / data / model-parallel / embedding groups.

MI355X-native equivalent of Megatron's ``megatron.core.parallel_state`` (the
reference's log shows rank 0 creating world/TP/PP/DP/MP communicators, NB3:1214, and
`megatron/data/gpt_dataset.py:462-469` all-reduces over the DP and PP groups).

Rank layout (identical to Megatron so checkpoints and logs line up): TP is the fastest-varying
dimension, then CP (context parallel, Megatron-core's order), then DP, then PP.
world = tp * cp * dp * pp.

    tp group : consecutive ranks                     e.g. TP2 PP2 DP2 -> {0,1} {2,3} {4,5} {6,7}
    cp group : same (pp, dp, tp), stride tp           (cp = 1: singletons)
    dp group : same (pp stage, cp rank, tp rank)                         {0,2} {1,3} {4,6} {5,7}
    dp_cp    : same (pp stage, tp rank) — the gradient-reduction group (CP ranks hold the same
               parameters and see different tokens, so their gradients are averaged like DP's)
    pp group : stride world/pp                                           {0,4} {1,5} {2,6} {3,7}

On one MI355X node every GPU pair has its own xGMI link (fully connected, no switch), so the
layout does not change link contention; it is kept for compatibility.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    tp: int = 1
    pp: int = 1
    dp: int = 1
    cp: int = 1
    rank: int = 0
    world: int = 1
    tp_group: object = None
    pp_group: object = None
    dp_group: object = None
    cp_group: object = None
    dp_cp_group: object = None       # gradient reduction over dp x cp (== dp_group when cp == 1)
    mp_group: object = None          # tp x pp (model-parallel)
    embd_group: object = None        # first + last pipeline stage (tied embeddings)
    tp_ranks: List[int] = field(default_factory=list)
    pp_ranks: List[int] = field(default_factory=list)
    dp_ranks: List[int] = field(default_factory=list)
    cp_ranks: List[int] = field(default_factory=list)
    dp_cp_ranks: List[int] = field(default_factory=list)
    embd_ranks: List[int] = field(default_factory=list)
    virtual_pp: Optional[int] = None
    virtual_pp_rank: int = 0

    # ---- ranks inside groups
    @property
    def tp_rank(self) -> int:
        return self.tp_ranks.index(self.rank) if self.tp_ranks else 0

    @property
    def pp_rank(self) -> int:
        return self.pp_ranks.index(self.rank) if self.pp_ranks else 0

    @property
    def dp_rank(self) -> int:
        return self.dp_ranks.index(self.rank) if self.dp_ranks else 0

    @property
    def cp_rank(self) -> int:
        return self.cp_ranks.index(self.rank) if self.cp_ranks else 0

    @property
    def dp_cp_rank(self) -> int:
        """Rank in the gradient-reduction (dp x cp) group: the ZeRO shard index."""
        return self.dp_cp_ranks.index(self.rank) if self.dp_cp_ranks else self.dp_rank

    def is_first_stage(self, ignore_virtual: bool = False) -> bool:
        if not ignore_virtual and self.virtual_pp is not None and self.virtual_pp_rank != 0:
            return False
        return self.pp_rank == 0

    def is_last_stage(self, ignore_virtual: bool = False) -> bool:
        if not ignore_virtual and self.virtual_pp is not None and self.virtual_pp_rank != self.virtual_pp - 1:
            return False
        return self.pp_rank == self.pp - 1

    @property
    def next_pp_rank(self) -> int:
        return self.pp_ranks[(self.pp_rank + 1) % self.pp]

    @property
    def prev_pp_rank(self) -> int:
        return self.pp_ranks[(self.pp_rank - 1) % self.pp]


_STATE: Optional[ParallelState] = None


def _new_group(ranks, backend=None):
    """Every rank calls this identically (single-rank groups are created too). RCCL groups get a
    high-priority internal stream (comm/streams.nccl_pg_options; SMDT_COMM_PRIORITY=normal: off):
    TP / SP exchanges, pipeline p2p and DP buckets overlap GEMMs and must not queue behind them."""
    kw = {}
    if (backend or dist.get_backend()) == "nccl":
        from ..comm.streams import nccl_pg_options
        opts = nccl_pg_options()
        if opts is not None:
            kw["pg_options"] = opts
    return dist.new_group(ranks, backend=backend, **kw)


def initialize_model_parallel(tensor_model_parallel_size: int = 1, pipeline_model_parallel_size: int = 1,
                              virtual_pipeline_model_parallel_size: Optional[int] = None,
                              context_parallel_size: int = 1) -> ParallelState:
    """Create every group. Must be called on all ranks after ``init_process_group``."""
    global _STATE
    tp, pp, cp = int(tensor_model_parallel_size), int(pipeline_model_parallel_size), int(context_parallel_size)
    if not dist.is_initialized():
        _STATE = ParallelState(tp=1, pp=1, dp=1, rank=0, world=1, tp_ranks=[0], pp_ranks=[0], dp_ranks=[0],
                               cp_ranks=[0], dp_cp_ranks=[0], embd_ranks=[0])
        if tp != 1 or pp != 1 or cp != 1:
            raise RuntimeError("model / context parallelism requires torch.distributed to be initialised")
        return _STATE
    world, rank = dist.get_world_size(), dist.get_rank()
    if world % (tp * pp * cp) != 0:
        raise RuntimeError(f"world size {world} not divisible by tp({tp}) * pp({pp}) * cp({cp})")
    dp = world // (tp * pp * cp)
    st = ParallelState(tp=tp, pp=pp, dp=dp, cp=cp, rank=rank, world=world,
                       virtual_pp=virtual_pipeline_model_parallel_size)
    stage = world // pp

    def rk(p, d, c, t):
        return p * stage + d * (tp * cp) + c * tp + t

    # data-parallel groups (same pp stage, cp rank, tp rank)
    for p in range(pp):
        for c in range(cp):
            for t in range(tp):
                ranks = [rk(p, d, c, t) for d in range(dp)]
                g = _new_group(ranks)
                if rank in ranks:
                    st.dp_group, st.dp_ranks = g, ranks
    # context-parallel groups (same pp, dp, tp) and the dp x cp gradient groups (same pp, tp)
    if cp > 1:
        for p in range(pp):
            for d in range(dp):
                for t in range(tp):
                    ranks = [rk(p, d, c, t) for c in range(cp)]
                    g = _new_group(ranks)
                    if rank in ranks:
                        st.cp_group, st.cp_ranks = g, ranks
        for p in range(pp):
            for t in range(tp):
                ranks = sorted(rk(p, d, c, t) for d in range(dp) for c in range(cp))
                g = _new_group(ranks)
                if rank in ranks:
                    st.dp_cp_group, st.dp_cp_ranks = g, ranks
    else:
        st.cp_ranks = [rank]
        st.dp_cp_group, st.dp_cp_ranks = st.dp_group, st.dp_ranks
    # tensor-parallel groups
    for i in range(world // tp):
        ranks = list(range(i * tp, (i + 1) * tp))
        g = _new_group(ranks)
        if rank in ranks:
            st.tp_group, st.tp_ranks = g, ranks
    # model-parallel (tp x pp) groups: same dp and cp index
    for d in range(dp):
        for c in range(cp):
            ranks = sorted(rk(p, d, c, t) for p in range(pp) for t in range(tp))
            g = _new_group(ranks)
            if rank in ranks:
                st.mp_group = g
    # pipeline groups + embedding groups
    for i in range(stage):
        ranks = list(range(i, world, stage))
        g = _new_group(ranks)
        if rank in ranks:
            st.pp_group, st.pp_ranks = g, ranks
        embd = [ranks[0], ranks[-1]] if len(ranks) > 1 else [ranks[0]]
        ge = _new_group(embd)
        if rank in embd:
            st.embd_group, st.embd_ranks = ge, embd
    _STATE = st
    st.initialized = True
    # xGMI IPC all-reduce for the TP group (SMDT_XGMI_ALLREDUCE=1; collective over the TP group)
    if tp > 1:
        from ..comm import xgmi
        st.tp_xgmi = xgmi.create_for_group(st.tp_group)
    # TP pairs exchange over every xGMI link of the node (collective over WORLD; kept only when
    # validated and measured faster than RCCL p2p, comm/relay.py)
    if tp == 2 and world in (4, 8):
        from ..comm import relay
        st.tp_relay = relay.create_for_pairs(st.tp_group)
    # TP groups of 4 / 8: sequence-parallel exchanges over all of the group's links (collective over
    # the TP group; kept only when measured faster than the ring, comm/tp_direct.py)
    if tp in (4, 8) and world in (4, 8):
        from ..comm import tp_direct
        st.tp_direct = tp_direct.create(st.tp_group)
    return st


def initialize_emulated_tensor_parallel(tensor_model_parallel_size: int = 1,
                                        data_parallel_size: int = 1) -> ParallelState:
    """ONE process as rank 0 of a ``tensor_model_parallel_size``-rank TP group and / or of a
    ``data_parallel_size``-rank DP group whose collectives are local stand-ins
    (comm/loopback.py): the per-rank work of a multi-GPU layout, timed on one GPU — bench.py
    --emulate-tp / benchmarks/predict_scaling.py (a TP rank's sharded compute), SMDT_EMULATE_DP
    for the SFT recipe (a ZeRO rank's 1/dp optimizer shard and its gradient reduce-scatter /
    parameter all-gather traffic on the receiving side). pp = 1; with tp > 1 the model-parallel
    group (grad-norm all-reduce) is the loopback group too. Timing only: never train with it."""
    global _STATE
    from ..comm.loopback import LoopbackGroup
    tp, dp = int(tensor_model_parallel_size), int(data_parallel_size)
    if dist.is_initialized() and dist.get_world_size() != 1:
        raise RuntimeError("TP / DP emulation runs in a single process (world size 1)")
    if not dist.is_initialized():     # a one-rank world: c10d's group calls need a default group
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo", store=dist.HashStore(),
                                rank=0, world_size=1)
    world_group = dist.group.WORLD
    tg = LoopbackGroup(tp) if tp > 1 else world_group
    dg = LoopbackGroup(dp) if dp > 1 else world_group
    st = ParallelState(tp=tp, pp=1, dp=dp, rank=0, world=1, tp_group=tg, mp_group=tg if tp > 1 else None,
                       dp_group=dg, dp_cp_group=dg, tp_ranks=list(range(tp)),
                       pp_ranks=[0], dp_ranks=list(range(dp)), cp_ranks=[0], dp_cp_ranks=list(range(dp)),
                       embd_ranks=[0])
    st.initialized = True
    st.emulated = True
    from ..comm.loopback import PacedDirectEngine, direct_standin
    ds = direct_standin()
    if ds is not None and tp not in (4, 8):
        import warnings
        warnings.warn(f"SMDT_LINK_STANDIN=direct models the TP4 / TP8 direct engine; at tp {tp} the "
                      "emulated exchanges stay in-line copies (use 'relay' or '<GB/s>:<workgroups>')")
    if ds is not None and tp in (4, 8):
        # the TP4 / TP8 exchanges through a paced stand-in of the direct multi-link engine
        from ..comm.tp_direct import TpDirect
        st.tp_direct = TpDirect(PacedDirectEngine(tp, *ds), tg, world=tp, rank=0)
    _STATE = st
    return st


def xgmi_engine(group):
    """The xGMI all-reduce engine bound to ``group`` (only the TP group has one), else None."""
    st = _STATE
    if st is None or group is None or group is not st.tp_group:
        return None
    return getattr(st, "tp_xgmi", None)


def model_parallel_is_initialized() -> bool:
    return _STATE is not None and getattr(_STATE, "initialized", False)


def get_state() -> ParallelState:
    global _STATE
    if _STATE is None:
        _STATE = ParallelState(tp_ranks=[0], pp_ranks=[0], dp_ranks=[0], cp_ranks=[0], dp_cp_ranks=[0],
                               embd_ranks=[0])
    return _STATE


def destroy_model_parallel():
    global _STATE
    _STATE = None


# Megatron-style accessors -------------------------------------------------------------------

def get_tensor_model_parallel_world_size() -> int:
    return get_state().tp


def get_tensor_model_parallel_rank() -> int:
    return get_state().tp_rank


def get_tensor_model_parallel_group():
    return get_state().tp_group


def get_pipeline_model_parallel_world_size() -> int:
    return get_state().pp


def get_pipeline_model_parallel_rank() -> int:
    return get_state().pp_rank


def get_data_parallel_world_size() -> int:
    return get_state().dp


def get_data_parallel_rank() -> int:
    return get_state().dp_rank


def get_data_parallel_group(with_context_parallel: bool = False):
    st = get_state()
    return st.dp_cp_group if with_context_parallel else st.dp_group


def get_context_parallel_world_size() -> int:
    return get_state().cp


def get_context_parallel_rank() -> int:
    return get_state().cp_rank


def get_context_parallel_group():
    return get_state().cp_group


def env_rank_info():
    """(rank, local_rank, world_size) from torchrun or the OMPI_COMM_WORLD_* contract
    (the reference's `pretrain_gpt.py:10-13` remaps OMPI -> torch env vars)."""
    def first(*names, default=None):
        for n in names:
            if n in os.environ:
                return int(os.environ[n])
        return default
    rank = first("RANK", "OMPI_COMM_WORLD_RANK", default=0)
    local = first("LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", default=0)
    world = first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", default=1)
    return rank, local, world
