"""Partitioned model construction for ZeRO-3 — the equivalent of DeepSpeed's ``zero.Init``.

The reference's Alpaca job builds OPT-125m under ZeRO-3 so that every rank materialises only its
partition of the weights while the model is being constructed ("num_elems = 0.16B" at load,
/root/reference/4_training_alpaca_deepspeed.ipynb:1580; DS config
configs/default_offload_opt_param.json:23-41). Here:

    with zero_init.Init(dp_group):
        model = HFCausalLM.from_pretrained(...)      # or any nn.Module constructor
    engine = ZeroEngine(model, ds_config)            # stage 3

Inside the context every parameter is cut when the constructor of the module that owns it
returns (as DeepSpeed's zero.Init, which wraps ``nn.Module.__init__``): a module's own
``reset_parameters()`` / init code therefore runs on the full tensor, then this rank keeps 1/dp of
its flattened elements (``p._zi_shard``) and the parameter's storage is released (a 0-element
placeholder; its logical shape is in ``p._zi_shape``). A rank never holds more than its shards plus
the parameters of the ONE module being constructed (a transformer block's own tensors, not the
model). A parameter assigned to a module outside of any constructor is cut at once. Code in a
PARENT's constructor that touches an already-built child's parameters (e.g. a post-init pass over
the whole model) must do so under ``gathered()``, exactly as with DeepSpeed. DistributedDataParallel lays out
its buckets from the logical shapes, and the stage-3 partitioner assembles its bucket shards from
these per-parameter shards with one all-gather per parameter (transient: a single parameter at a
time), so the full model never exists on any rank (parallel/zero3.py).

Parameters are initialised exactly as without the context (the construction runs unchanged; only
the storage is cut afterwards), so a partitioned build trains bit-identically to a resident one.
Code that reads or writes a partitioned parameter's values afterwards (checkpoint loading, the
recipe's embedding resize) uses ``gathered([...])`` — DeepSpeed's ``GatheredParameters``: the full
value exists inside the block and the block's changes are cut back into the shards on exit — or
``load_full_`` to set a parameter from a full tensor without any gather.
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.distributed as dist
import torch.nn as nn


def is_partitioned(p) -> bool:
    return hasattr(p, "_zi_shape")


def logical_shape(p):
    return tuple(p._zi_shape) if is_partitioned(p) else tuple(p.shape)


def logical_numel(p) -> int:
    return int(math.prod(p._zi_shape)) if is_partitioned(p) else p.numel()


class Init:
    """Context manager: parameters built inside are partitioned over ``dp_group`` as soon as the
    constructor of the module that owns them returns (see the module docstring)."""

    def __init__(self, dp_group=None, enabled: bool = True):
        self.enabled = bool(enabled)
        self.group = dp_group
        self.dp = dist.get_world_size(dp_group) if (dist.is_initialized() and enabled) else 1
        self.rank = dist.get_rank(dp_group) if self.dp > 1 else 0
        self.shard_bytes = 0          # bytes of shards kept so far
        self.peak_bytes = 0           # max of shards kept + full parameters not yet cut
        self.largest_param_bytes = 0
        self.params = 0
        self._pending = {}            # id -> bytes of full parameters waiting for their constructor
        self._orig = None

    def __enter__(self):
        if not self.enabled:
            return self
        self._orig = nn.Module.register_parameter
        orig, me = self._orig, self

        def register_parameter(mod, name, param):
            orig(mod, name, param)
            # inside a constructor of ``mod``: cut when the outermost one returns (its init code
            # still has to write the full tensor); otherwise now
            if mod.__dict__.get("_zi_init_depth", 0) == 0:
                me._maybe_partition(param)
            elif param is not None and param.device.type != "meta" and not is_partitioned(param):
                me._pending[id(param)] = (param.numel() * param.element_size(), id(mod))
                me.peak_bytes = max(me.peak_bytes, me.shard_bytes + me._waiting())
        nn.Module.register_parameter = register_parameter
        self._wrapped = {}
        for cls in _module_classes():
            self._wrap_init(cls)

        # chain to (and on exit restore) whatever __init_subclass__ nn.Module had: an outer Init
        # context's hook, or another library's
        self._prev_init_subclass = prev = nn.Module.__dict__.get("__init_subclass__")

        def init_subclass(cls, **kw):     # classes defined inside the context
            if prev is not None:
                prev.__get__(None, cls)(**kw)
            me._wrap_init(cls)
        nn.Module.__init_subclass__ = classmethod(init_subclass)
        return self

    def __exit__(self, *exc):
        if self._orig is not None:
            nn.Module.register_parameter = self._orig
            self._orig = None
            for cls, init in self._wrapped.items():
                cls.__init__ = init
            self._wrapped = {}
            if self._prev_init_subclass is not None:
                nn.Module.__init_subclass__ = self._prev_init_subclass
            else:
                del nn.Module.__init_subclass__
            self._prev_init_subclass = None
        return False

    def _wrap_init(self, cls):
        init = cls.__dict__.get("__init__")
        if init is None or cls in self._wrapped:
            return
        me = self

        def __init__(mod, *args, **kwargs):
            depth = mod.__dict__.get("_zi_init_depth", 0)
            object.__setattr__(mod, "_zi_init_depth", depth + 1)
            try:
                init(mod, *args, **kwargs)
            finally:
                object.__setattr__(mod, "_zi_init_depth", depth)
            if depth == 0:      # the outermost constructor of this object returned
                mod.__dict__.pop("_zi_init_depth", None)
                for p in mod.__dict__.get("_parameters", {}).values():
                    me._maybe_partition(p)
                for k in [k for k, v in me._pending.items() if v[1] == id(mod)]:
                    del me._pending[k]        # replaced before the constructor returned
        __init__.__wrapped__ = init
        self._wrapped[cls] = init
        cls.__init__ = __init__

    def _waiting(self):
        return sum(v[0] for v in self._pending.values())

    def _maybe_partition(self, p):
        if p is not None and not is_partitioned(p) and p.numel() > 0 and p.device.type != "meta":
            self._partition(p)

    @torch.no_grad()
    def _partition(self, p: nn.Parameter):
        full_bytes = p.numel() * p.element_size()
        waiting = self._waiting() + (0 if id(p) in self._pending else full_bytes)
        self.peak_bytes = max(self.peak_bytes, self.shard_bytes + waiting)
        self.largest_param_bytes = max(self.largest_param_bytes, full_bytes)
        _cut(p, self.dp, self.rank, self.group)
        self._pending.pop(id(p), None)
        self.shard_bytes += p._zi_shard.numel() * p._zi_shard.element_size()
        self.params += 1


def _module_classes():
    """nn.Module and every subclass defined so far."""
    out, todo = [], [nn.Module]
    while todo:
        c = todo.pop()
        out.append(c)
        todo.extend(c.__subclasses__())
    return list(dict.fromkeys(out))


def _group_dims(group):
    dp = dist.get_world_size(group) if dist.is_initialized() else 1
    return dp, (dist.get_rank(group) if dp > 1 else 0)


@torch.no_grad()
def _cut(p, dp: int, rank: int, group, full=None):
    """Keep this rank's 1/dp of ``full`` (default: p's own data) as p's shard; placeholder data."""
    shape = tuple(p.shape) if full is None else tuple(full.shape)
    flat = (p.data if full is None else full).reshape(-1)
    n = flat.numel()
    c = (n + dp - 1) // dp
    shard = torch.zeros(c, dtype=p.dtype, device=p.device)
    lo, hi = min(n, rank * c), min(n, (rank + 1) * c)
    shard[:hi - lo].copy_(flat[lo:hi])
    p._zi_shape = shape
    p._zi_shard = shard
    p._zi_group = group
    p.data = torch.empty(0, dtype=p.dtype, device=p.device)


@torch.no_grad()
def gather_full(p, group=None) -> torch.Tensor:
    """The flattened full value of a partitioned parameter over ``group`` (one all-gather;
    transient). ``group`` must have the size the parameter was partitioned for."""
    n = logical_numel(p)
    shard = p._zi_shard
    dp = dist.get_world_size(group) if dist.is_initialized() else 1
    if shard.numel() != (n + dp - 1) // dp:
        raise ValueError(f"a parameter partitioned for another group size cannot be gathered over {dp} ranks")
    if dp == 1:
        return shard[:n]
    out = torch.empty(dp * shard.numel(), dtype=shard.dtype, device=shard.device)
    dist.all_gather_into_tensor(out, shard, group=group)
    return out[:n]


@torch.no_grad()
def load_full_(p, value: torch.Tensor):
    """Set a parameter from its full value (every rank passes the same tensor; no collective)."""
    if not is_partitioned(p):
        p.data.copy_(value.to(p.dtype))
        return
    if tuple(value.shape) != logical_shape(p):
        raise ValueError(f"shape {tuple(value.shape)} != {logical_shape(p)}")
    _cut(p, *_group_dims(p._zi_group), p._zi_group, full=value.to(p.dtype))


@contextlib.contextmanager
def gathered(params, group=None):
    """Collective: inside the block the partitioned ones among ``params`` hold their full value
    (``p.data`` with the logical shape); on exit whatever the block wrote is cut back into the
    shards. Every rank of the group must enter with the same parameters."""
    ps = [p for p in dict.fromkeys(params) if p is not None and is_partitioned(p)]
    for p in ps:
        g = p._zi_group if group is None else group
        p.data = gather_full(p, g).view(p._zi_shape).clone()
        del p._zi_shard
        del p._zi_shape
    try:
        yield
    finally:
        for p in ps:
            g = p._zi_group if group is None else group
            _cut(p, *_group_dims(g), g)


def cast_(p, dtype):
    """Cast a partitioned parameter's shard (and placeholder) to ``dtype``."""
    p._zi_shard = p._zi_shard.to(dtype)
    p.data = torch.empty(0, dtype=dtype, device=p.device)
