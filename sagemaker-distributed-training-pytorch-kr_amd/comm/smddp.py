"""``smddp`` process-group backend for unmodified SageMaker data-parallel scripts.

The reference's DDP recipes do ``import smdistributed.dataparallel.torch.torch_smddp`` and then
``dist.init_process_group(backend="smddp")`` (/root/reference/1_training_mnist_ddp/
pytorch_mnist_ddp.py:89-90, /root/reference/2_training_oxford-pet_ddp/pytorch_oxford_ddp.py:206-211)
and wrap the model in ``torch.nn.parallel.DistributedDataParallel``, whose bucket all-reduces then
run on SMDDP's own all-reduce (NB2:387-404 logs its "balanced fusion buffers").

Importing this module registers the same backend name. Its process group is a real backend, not
an alias: ``SMDDPProcessGroup`` owns an RCCL group (ProcessGroupNCCL; on ROCm that IS RCCL over
xGMI) — or Gloo for CPU tensors — and routes

* GPU ``allreduce`` (SUM / AVG, one dense contiguous fp32 / bf16 / fp16 tensor, 16-byte multiple,
  2 / 4 / 8 ranks on one node) through the single-launch xGMI all-reduce engine
  (``comm/xgmi.py``: every peer read over its own link, one-shot below and two-shot above
  ``ONE_SHOT_MAX_BYTES``, fp32 accumulation in rank order so every rank gets identical bits).
  The engine is built collectively on the first eligible call, validated against RCCL and timed
  per op, and kept only for the ops it wins on this node. Each all-reduce runs on the ENGINE'S
  stream, ordered after the caller's work so far, and the returned Work carries a CUDA future
  completed by an event on that stream: torch DDP's reducer keeps launching backward kernels on
  the compute stream while the bucket travels, and its ``wait()`` at the end of backward is a
  device-side stream wait (no host block) — the overlap that RCCL's own stream gives. Every
  ``CHECK_EVERY`` engine calls the ranks agree on the engine's sticky error word WITHOUT a host
  synchronisation in the hook path: the MAX all-reduce is issued on RCCL and copied to pinned
  memory by a side stream, and that flag is read at the next check, ``CHECK_EVERY`` calls later
  (every rank at the same call, so every rank decides alike). A peer that never arrived turns the
  path off on every rank for the rest of the run, with a warning, and RCCL takes over;
* every other collective straight to RCCL (GPU tensors) or to a host Gloo group (CPU tensors,
  e.g. object collectives), created on first use.

SMDDP's parameter-server all-reduce exists to use EFA across p3 / p4 nodes; inside one
xGMI-connected node the peer-read all-reduce (small messages) and RCCL's rings (large ones) are the
right algorithms, chosen per message size at run time. ``smddp_stats()`` reports how many calls
and bytes took each path (the per-collective metrics of SURVEY §5.5).
"""
from __future__ import annotations

import datetime
import os
import threading

import torch
import torch.distributed as dist

BACKEND = "smddp"
_REGISTERED = False
_STATS = {"xgmi_calls": 0, "xgmi_bytes": 0, "rccl_calls": 0, "rccl_bytes": 0}
# (start, end) CUDA events of engine all-reduces while comm stats are on (tests / profiling: where
# and when the bucket all-reduces ran)
_TIMINGS: list = []
CHECK_EVERY = 64   # engine all-reduces between two agreed error-word checks (one host sync each)


def smddp_stats() -> dict:
    """Calls / bytes of this process's smddp all-reduces per path (xgmi engine vs RCCL / Gloo)."""
    return dict(_STATS)


def _done_work(result):
    """A Work whose future already holds ``result`` (the engine ran on the current stream)."""
    from torch._C._distributed_c10d import _create_work_from_future
    fut = torch.futures.Future()
    fut.set_result(result)
    return _create_work_from_future(fut)


def _stream_work(result, stream):
    """A Work whose CUDA future completes on ``stream``: set inside that stream, the future records
    an event there, and ``wait()`` / ``then()`` make the waiter's CURRENT stream wait for it (a
    device-side dependency; the host never blocks)."""
    from torch._C._distributed_c10d import _create_work_from_future
    dev = result[0].device
    fut = torch.futures.Future(devices=[dev])
    with torch.cuda.stream(stream):
        fut.set_result(result)
    return _create_work_from_future(fut)


class SMDDPProcessGroup(dist.ProcessGroup):
    """The ``smddp`` backend object (see the module docstring)."""

    def __init__(self, store, rank: int, size: int, timeout):
        super().__init__(rank, size)
        timeout = timeout if isinstance(timeout, datetime.timedelta) else datetime.timedelta(seconds=float(timeout))
        # SMDT_SMDDP_INNER=gloo: Gloo underneath even with a GPU (multi-process tests that share
        # one GPU, where RCCL refuses two ranks on one device; the xGMI engine then runs over
        # same-device IPC mappings without its RCCL validation / timing)
        self._host_inner = not torch.cuda.is_available() or os.environ.get("SMDT_SMDDP_INNER") == "gloo"
        if not self._host_inner:
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = timeout
            self._inner = dist.ProcessGroupNCCL(store, rank, size, opts)
        else:
            opts = dist.ProcessGroupGloo._Options()
            opts._timeout = timeout
            opts._devices = [dist.ProcessGroupGloo.create_default_device()]
            self._inner = dist.ProcessGroupGloo(store, rank, size, opts)
        self._store, self._timeout, self._cpu = store, timeout, None
        self._engine = None
        self._state = "unset"       # unset -> building -> ready | off
        self._lock = threading.Lock()
        self._pending = None        # (event, pinned flag) of the last error-word check
        self._side = None

    def getBackendName(self) -> str:
        return BACKEND

    def _route(self, args):
        """RCCL for GPU tensors; a Gloo group (created on first use, collectively: every rank
        issues the same collectives) for CPU tensors, e.g. object collectives on host buffers."""
        t = _first_tensor(args)
        if t is None or t.is_cuda or self._host_inner:
            return self._inner
        if self._cpu is None:
            opts = dist.ProcessGroupGloo._Options()
            opts._timeout = self._timeout
            opts._devices = [dist.ProcessGroupGloo.create_default_device()]
            self._cpu = dist.ProcessGroupGloo(dist.PrefixStore("smddp_cpu", self._store), self.rank(), self.size(), opts)
        return self._cpu

    # ---- xGMI all-reduce path ----------------------------------------------------------------
    def _world_group(self):
        """The dist-level handle of this backend when it is the default (world) group — the only
        group SMDDP scripts use; subgroups stay on RCCL."""
        try:
            if dist.get_world_size() == self.size() and dist.get_rank() == self.rank():
                return dist.group.WORLD
        except (RuntimeError, ValueError):
            pass
        return None

    def _xgmi(self, t: torch.Tensor):
        if self._state == "off" or self._state == "building":
            return None
        if self._state == "unset":
            from . import xgmi
            if not (t.is_cuda and self.size() in (2, 4, 8)) or xgmi.explicitly_off():
                self._state = "off"
                return None
            group = self._world_group()
            if group is None:
                self._state = "off"
                return None
            with self._lock:
                self._state = "building"   # the engine's own set-up collectives go to RCCL
                try:
                    if self._host_inner:
                        self._engine = xgmi.XgmiAllReduce(group, region_bytes=8 << 20, blocks=32, validate=False)
                    else:
                        self._engine = xgmi.create_for_group(group, auto=True, tune=True, log=print)
                finally:
                    self._state = "ready" if self._engine is not None else "off"
        eng = self._engine
        if eng is None or not eng.active:
            return None
        return eng

    def _check(self, eng, dev):
        """Every ``CHECK_EVERY`` engine calls (the same call on every rank): read the agreed flag of
        the previous check — issued ``CHECK_EVERY`` calls ago, so its event has long completed and
        reading it does not stall — then issue this one: MAX of the sticky error words over the
        group on the inner group (async), copied to pinned memory by a side stream."""
        pend, self._pending = self._pending, None
        if pend is not None:
            ev, pinned = pend
            if ev is not None:
                ev.synchronize()
            if int(pinned[0]) > 0:
                import warnings
                warnings.warn("smddp: an xGMI all-reduce timed out waiting for a peer (its output was NaN-filled); "
                              "all later all-reduces of this group run on RCCL")
                eng.deactivate("peer timeout")
                self._state = "off"
                return
        flag = (eng.error_tensor() != 0).to(torch.int32).view(1).to(dev)
        mx = dist.AllreduceOptions()
        mx.reduceOp = dist.ReduceOp.MAX
        if self._host_inner:             # (tests sharing one GPU: Gloo underneath)
            self._inner.allreduce([flag], mx).wait()
            self._pending = (None, flag.cpu())
            return
        work = self._inner.allreduce([flag], mx)
        if self._side is None:
            from .streams import comm_stream
            self._side = comm_stream(dev)
        pinned = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        with torch.cuda.stream(self._side):
            work.wait()                  # the side stream waits for RCCL, not the compute stream
            pinned.copy_(flag, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self._side)
        flag.record_stream(self._side)
        self._pending = (ev, pinned)

    def allreduce(self, tensors, opts=None):
        opts = opts if opts is not None else dist.AllreduceOptions()
        if len(tensors) == 1 and tensors[0].is_cuda:
            t = tensors[0]
            op = opts.reduceOp
            kind = "sum" if op == dist.ReduceOp.SUM else ("avg" if op == dist.ReduceOp.AVG else None)
            if kind is not None:
                from . import xgmi
                eng = self._xgmi(t) if xgmi.eligible(t, self.size()) else None
                h = eng.all_reduce_async(t, kind) if eng is not None else None
                if h is not None:
                    _STATS["xgmi_calls"] += 1
                    _STATS["xgmi_bytes"] += t.numel() * t.element_size()
                    if h.start is not None:
                        _TIMINGS.append((h.start, h.event))
                    work = _stream_work(tensors, eng._stream)
                    if _STATS["xgmi_calls"] % CHECK_EVERY == 0:
                        self._check(eng, t.device)
                    return work
        _STATS["rccl_calls"] += 1
        _STATS["rccl_bytes"] += sum(x.numel() * x.element_size() for x in tensors)
        return self._route(tensors).allreduce(tensors, opts)


def _first_tensor(x):
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, (list, tuple)):
        for v in x:
            t = _first_tensor(v)
            if t is not None:
                return t
    return None


def _delegate(name):
    def f(self, *args, **kwargs):
        return getattr(self._route(args), name)(*args, **kwargs)
    f.__name__ = name
    f.__doc__ = f"``{name}`` on the RCCL group (GPU tensors) or the host Gloo group (CPU tensors)."
    return f


for _name in ("allreduce_coalesced", "allgather", "_allgather_base", "allgather_coalesced",
              "allgather_into_tensor_coalesced", "alltoall", "alltoall_base", "barrier", "broadcast", "gather",
              "recv", "recv_anysource", "reduce", "reduce_scatter", "_reduce_scatter_base",
              "reduce_scatter_tensor_coalesced", "scatter", "send", "monitored_barrier"):
    setattr(SMDDPProcessGroup, _name, _delegate(_name))


def DistributedDataParallel(module, *args, bucket_cap_mb=None, process_group=None, **kwargs):
    """``smdistributed.dataparallel.torch.parallel.DistributedDataParallel``: torch DDP whose
    gradient buckets ("fusion buffers") are sized for this node's links — comm/buckets.py's 8-32 MB
    from a start-up latency / bandwidth timing of the group's reduce-scatter, at least 4 buckets
    per rank so the first all-reduce starts early in backward — instead of torch's fixed 25 MB.
    An explicit ``bucket_cap_mb`` wins. Collective over the group (the timing)."""
    from . import buckets
    if bucket_cap_mb is None:
        ps = [p for p in module.parameters() if p.requires_grad]
        total = sum(p.numel() for p in ps)
        esz = ps[0].element_size() if ps else 4
        bucket_cap_mb = buckets.auto_bucket_elems(process_group or dist.group.WORLD, total, esz) * esz / 2 ** 20
    return torch.nn.parallel.DistributedDataParallel(module, *args, bucket_cap_mb=bucket_cap_mb,
                                                     process_group=process_group, **kwargs)


def _create(store, rank, size, timeout):
    return SMDDPProcessGroup(store, rank, size, timeout)


def register():
    global _REGISTERED
    if _REGISTERED or BACKEND in dist.Backend.backend_list:
        _REGISTERED = True
        return
    dist.Backend.register_backend(BACKEND, _create, devices=["cuda", "cpu"])
    _REGISTERED = True


register()
