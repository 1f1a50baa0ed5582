"""Single-node all-reduce over xGMI peer memory — the MI355X-native counterpart of SMDDP's fused
all-reduce and of NCCL's intra-node P2P path (SURVEY C2', C4, §5.8, §7.4 item 1).

Every rank allocates one staging buffer (4 regions: two call-parity halves x {input copy,
reduced slice}) and one uncached signal buffer, exports both with ``hipIpcGetMemHandle`` and maps
every peer's with ``hipIpcOpenMemHandle`` (dmabuf IPC on this ROCm). One kernel
(``csrc/kernels/xgmi_allreduce.hip``) then reads all 7 peers over their own xGMI links at once:

* one-shot (message <= ``ONE_SHOT_MAX_BYTES[world]``): every rank reduces the whole tensor;
* two-shot: reduce-scatter through peer reads, then an all-gather of the reduced slices;
* reduce-scatter / all-gather (ZeRO gradient shards and parameter gathers): one barrier, each link
  carries 1/W of the message;

reductions accumulate in fp32 in rank order, so every rank gets bit-identical results. Messages
larger than the staging region run as a sequence of region-sized calls (an all-reduce in flat
pieces, a reduce-scatter / all-gather in column bands of every slice). Anything the kernel does not
take — sizes that are not a multiple of 16 bytes, non-contiguous or CPU tensors, groups that span
hosts or are not 2 / 4 / 8 ranks — goes to RCCL unchanged.

The reference has no custom all-reduce (stock NCCL / SMDDP collectives). Its TP
all-reduces are 18.9 MB each (NB3) and its MNIST gradients 4.8 MB — the message range
this path is for. It is used by the tensor-parallel layers (sync all-reduces) and by the DDP
reducer (bucket all-reduces, ZeRO reduce-scatters and parameter all-gathers) when
``SMDT_XGMI_ALLREDUCE=1`` or when the job asked for the ``smddp`` backend — through
``init_distributed("smddp")`` or a direct ``dist.init_process_group(backend="smddp")``
(``SMDT_XGMI_ALLREDUCE=0`` turns it off).

An engine's calls must be issued in the same order on every rank of its group and on ONE stream
(the kernel double-buffers on a per-call counter); separate engines are used per group / stream.
"""
from __future__ import annotations

import os
import socket
import time
import warnings
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from . import health

# One-shot reads (W-1) full copies per rank; two-shot moves 2/W of the message per link but pays a
# second barrier. Crossover chosen for 7 x ~64 GB/s-per-direction links vs ~5 us per barrier.
ONE_SHOT_MAX_BYTES = {2: 4 << 20, 4: 1 << 20, 8: 512 << 10}
DEFAULT_REGION_BYTES = 64 << 20
DEFAULT_BLOCKS = 128

_SMDDP_REQUESTED = False
TUNED: Dict[str, dict] = {}  # run-time RCCL-vs-kernel timings of auto-mode engines (bench JSON)


def note_smddp_requested():
    """Called by ``init_distributed`` when a script asked for ``backend="smddp"``."""
    global _SMDDP_REQUESTED
    _SMDDP_REQUESTED = True


def explicitly_off() -> bool:
    return os.environ.get("SMDT_XGMI_ALLREDUCE") == "0"


def wanted(group=None) -> bool:
    v = os.environ.get("SMDT_XGMI_ALLREDUCE")
    if v is not None:
        return v == "1"
    if _SMDDP_REQUESTED:
        return True
    # a script that called dist.init_process_group(backend="smddp") directly
    try:
        return dist.is_initialized() and dist.get_backend(group) == "smddp"
    except (RuntimeError, ValueError):
        return False


def rccl_backend(group=None) -> bool:
    """True when ``group``'s collectives run on RCCL (``nccl``, or the ``smddp`` alias of it)."""
    try:
        return dist.get_backend(group) in ("nccl", "smddp")
    except (RuntimeError, ValueError):
        return False


def choose_algorithm(nbytes: int, world: int) -> str:
    return "one_shot" if nbytes <= ONE_SHOT_MAX_BYTES.get(world, 0) else "two_shot"


_MODE = {"one_shot": 0, "two_shot": 1, "reduce_scatter": 2, "all_gather": 3}


def eligible(t: torch.Tensor, world: int, region_bytes: int = 0) -> bool:
    """A tensor the kernel takes (any size: larger messages are chunked by the engine)."""
    nbytes = t.numel() * t.element_size()
    return (t.is_cuda and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and world in (2, 4, 8) and 0 < nbytes and nbytes % 16 == 0 and t.data_ptr() % 16 == 0)


def _bands(n: int, per_call: int, align: int):
    """[lo, hi) pieces of [0, n), each at most ``per_call`` and (but the last) a multiple of align."""
    step = max(align, per_call // align * align)
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


def _timing_event(stream):
    """A start event on ``stream`` when per-collective stats are being collected, else None."""
    from . import stats
    if not stats.active():
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record(stream)
    return ev


class _EventHandle:
    """``work.wait()``-compatible handle of a call issued on the engine's side stream."""

    def __init__(self, event, start=None):
        self.event = event
        self.start = start          # recorded before the call when comm stats are on

    def timing(self):
        """(start, end) events of the call for comm/stats.py, or None."""
        return (self.start, self.event) if self.start is not None else None

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)
        return True

    def is_completed(self):
        return self.event.query()


class IpcEngine:
    """Shared plumbing of the xGMI engines: every rank of ``group`` (None = WORLD) allocates its
    buffers (``specs`` = [(bytes, uncached)]), exports them with hipIpcGetMemHandle and maps every
    peer's; ``ptrs[i][r]`` is buffer i of rank r as seen from this process. Construction and
    ``close`` are collective over the group, and every rank reaches the same verdict."""

    def _setup_ipc(self, group, specs):
        self.C = _ext.ext()
        self._ipc_group = group
        self._own: List[int] = []
        self._opened: List[int] = []
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname(), group=group)
        if len(set(hosts)) != 1:
            raise RuntimeError(f"xGMI engines need every rank of the group on one node, got {sorted(set(hosts))}")
        err = None
        try:
            for nbytes, uncached in specs:
                self._own.append(self.C.ipc_malloc(int(nbytes), bool(uncached)))
            mine = tuple(self.C.ipc_get_handle(p) for p in self._own)
        except RuntimeError as e:  # still take part in the collectives below
            err, mine = e, None
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        ptrs: List[List[int]] = [[] for _ in specs]
        if err is None and all(h is not None for h in handles):
            try:
                for r, hs in enumerate(handles):
                    for i, h in enumerate(hs):
                        if r == rank:
                            ptrs[i].append(self._own[i])
                        else:
                            p = self.C.ipc_open(h)
                            self._opened.append(p)
                            ptrs[i].append(p)
            except RuntimeError as e:
                err = e
        if not self._agree(err is None):
            self._close_ipc()
            raise RuntimeError(f"xGMI IPC setup failed on some rank ({err!r} here)")
        return ptrs

    _WORD_OFFSET = "ar_word_offset"

    def _word(self, which: int) -> torch.Tensor:
        """Word ``which`` (0 sticky error, 1 spin limit) of this rank's signal buffer, as a device
        tensor aliasing the uncached memory."""
        return self.C.signal_word(self._sig, getattr(self.C, self._WORD_OFFSET)(which))

    def error_tensor(self) -> torch.Tensor:
        if getattr(self, "_err_t", None) is None:
            self._err_t = self._word(0)
        return self._err_t

    def set_spin_limit(self, polls: int):
        """Polls of a peer flag before a wait gives up (0: the kernel default, ~seconds). Tests lower
        it to inject a timeout."""
        self._word(1).fill_(int(polls))
        torch.cuda.synchronize()

    def deactivate(self, reason: str = ""):
        """Stop taking calls (callers fall back to RCCL); buffers stay mapped until ``close``."""
        self.active = False
        self.deactivated = reason or "deactivated"

    def _agree(self, ok: bool) -> bool:
        # gloo groups (multi-process tests on one GPU) agree on the host; RCCL on the device
        on_host = dist.get_backend(self._ipc_group) == "gloo"
        dev = torch.device("cpu") if on_host else torch.device("cuda", torch.cuda.current_device())
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self._ipc_group)
        return bool(flag.item())

    def _close_ipc(self):
        """Collective: unmap the peers' buffers, then free this rank's own."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if dist.is_initialized():
            dist.barrier(group=self._ipc_group)
        for p in self._opened:
            try:
                self.C.ipc_close(p)
            except RuntimeError:  # pragma: no cover
                pass
        self._opened = []
        if dist.is_initialized():
            dist.barrier(group=self._ipc_group)
        for p in self._own:
            self.C.ipc_free(p)
        self._own = []


class XgmiAllReduce(IpcEngine):
    """All-reduce engine for one process group whose ranks share a node (one GPU per rank)."""

    def __init__(self, group=None, region_bytes: int = DEFAULT_REGION_BYTES, blocks: int = DEFAULT_BLOCKS,
                 validate: bool = True):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if self.world not in (2, 4, 8):
            raise ValueError(f"xGMI all-reduce supports 2, 4 or 8 ranks, not {self.world}")
        self.region = (int(region_bytes) + 4095) // 4096 * 4096
        self.blocks = int(blocks)
        # ops this engine takes; ``tune`` turns off the ones RCCL does faster on this node
        self.use = {"all_reduce": True, "reduce_scatter": True, "all_gather": True}
        self.calls = 0
        self.bytes_moved = 0
        self._stream = None
        self.active = False
        self._sig = None
        self.data_ptrs, self.sig_ptrs = self._setup_ipc(group, [(4 * self.region, False),
                                                                (_ext.ext().ar_signal_bytes(), True)])
        self._sig = self.sig_ptrs[self.rank]
        self.active = True
        if validate and not self._validate():
            self.close()
            raise RuntimeError("xGMI all-reduce failed its validation against RCCL")
        health.register(self)

    # ------------------------------------------------------------------ helpers
    VALIDATE_BUCKET_BYTES = 32 << 20     # the largest DP bucket comm/buckets.py picks

    def _validate(self) -> bool:
        """Exact check against RCCL on integer-valued data (order-independent sums) at the sizes
        and modes training sends: one-shot and two-shot all-reduce (twice, both buffer halves), an
        all-reduce 1.5x the staging region (chunked), and an fp32 reduce-scatter (in place, the
        ZeRO pattern) plus a bf16 all-gather at the largest gradient-bucket size, which cross a
        region band when the region is smaller than the bucket."""
        dev = torch.device("cuda", torch.cuda.current_device())
        W, good = self.world, True
        n2 = ONE_SHOT_MAX_BYTES[W] // 4 * 2 + 1024
        big = self.region * 3 // 2 // 4 // 16 * 16 + 16
        for n, reps in ((4096, 2), (min(n2, self.region // 4), 2), (big, 1)):
            for rep in range(reps):
                x = (torch.arange(n, device=dev, dtype=torch.float32) % 97) + 1000.0 * self.rank + rep
                ref = x.clone()
                dist.all_reduce(ref, group=self.group)
                self.all_reduce(x)
                good &= bool(torch.equal(x, ref))
        ns = self.VALIDATE_BUCKET_BYTES // 4 // W // 64 * 64
        full = (torch.arange(W * ns, device=dev, dtype=torch.float32) % 89) + 7.0 * self.rank
        want = full.clone()
        dist.all_reduce(want, group=self.group)
        mine = full.view(W, ns)[self.rank]
        if self.reduce_scatter(mine, full):
            good &= bool(torch.equal(mine, want.view(W, ns)[self.rank]))
        nb = self.VALIDATE_BUCKET_BYTES // 2 // W // 64 * 64
        part = ((torch.arange(nb, device=dev, dtype=torch.float32) % 251) + 256.0 * self.rank).to(torch.bfloat16)
        ref_ag = torch.empty(W * nb, device=dev, dtype=torch.bfloat16)
        dist.all_gather_into_tensor(ref_ag, part, group=self.group)
        got = torch.empty_like(ref_ag)
        if self.all_gather(got, part):
            good &= bool(torch.equal(got, ref_ag))
        torch.cuda.synchronize()
        good &= self.error() == 0
        return self._agree(good)

    def tune(self, nbytes: int = 32 << 20, iters: int = 8) -> Dict[str, tuple]:
        """Time every op against RCCL at ``nbytes`` (bf16) on this group's real links and keep
        only those where the kernel is faster on every rank. Returns {op: (rccl_ms, xgmi_ms,
        rccl_busbw_GBps, xgmi_busbw_GBps)} (times: max over ranks)."""
        W = self.world
        dev = torch.device("cuda", torch.cuda.current_device())
        n = max(W * 8, nbytes // 2 // (W * 8) * (W * 8))
        full = torch.randn(n, device=dev, dtype=torch.bfloat16)
        part = torch.empty(n // W, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(full)
        g = self.group
        if dist.get_backend(g) == "gloo":  # multi-process tests on one GPU: host-side reference ops
            def ref_ar():
                dist.all_reduce(full.cpu(), group=g)

            def ref_rs():
                c = full.cpu()
                dist.all_reduce(c, group=g)
                part.copy_(c.view(W, -1)[self.rank])

            def ref_ag():
                lst = [torch.empty(part.shape, dtype=part.dtype) for _ in range(W)]
                dist.all_gather(lst, part.cpu(), group=g)
                out.copy_(torch.cat(lst))
        else:
            def ref_ar():
                dist.all_reduce(full, group=g)

            def ref_rs():
                dist.reduce_scatter_tensor(part, full, group=g)

            def ref_ag():
                dist.all_gather_into_tensor(out, part, group=g)
        cases = {
            "all_reduce": (ref_ar, lambda: self.all_reduce(full), 2.0 * (W - 1) / W),
            "reduce_scatter": (ref_rs, lambda: self.reduce_scatter(part, full), (W - 1) / W),
            "all_gather": (ref_ag, lambda: self.all_gather(out, part), (W - 1) / W),
        }
        res = {}
        for op, (ref_fn, our_fn, factor) in cases.items():
            ts = []
            for fn in (ref_fn, our_fn):
                for _ in range(2):
                    fn()
                torch.cuda.synchronize()
                dist.barrier(group=self.group)
                t0 = time.perf_counter()
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                t = torch.tensor([(time.perf_counter() - t0) / iters],
                                 device="cpu" if dist.get_backend(g) == "gloo" else dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX, group=g)
                ts.append(float(t.item()))
            self.use[op] = ts[1] < ts[0]
            res[op] = (ts[0] * 1e3, ts[1] * 1e3, n * 2 * factor / ts[0] / 1e9, n * 2 * factor / ts[1] / 1e9)
        self.check()
        return res

    # ------------------------------------------------------------------ API
    def fits(self, t: torch.Tensor) -> bool:
        return self.active and eligible(t, self.world, self.region)

    def _call(self, mode: str, inp: torch.Tensor, out: torch.Tensor, n: int, slice_stride: int, scale: float):
        self.C.xgmi_collective(_MODE[mode], inp, out, self.data_ptrs, self.sig_ptrs, self.rank, 1, self.region,
                               self.blocks, n, slice_stride, scale)
        self.calls += 1
        self.bytes_moved += n * inp.element_size() * (self.world if mode in ("reduce_scatter", "all_gather") else 1)

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> bool:
        """In-place all-reduce of ``t`` on the current stream (region-sized pieces); False
        (nothing done) when the tensor is not eligible, so the caller falls back to RCCL."""
        if not (self.use["all_reduce"] and self.fits(t)):
            return False
        scale = 1.0 / self.world if op == "avg" else 1.0
        flat = t.view(-1)
        per = self.region // t.element_size()
        for lo, hi in _bands(flat.numel(), per, 16 // t.element_size()):
            piece = flat[lo:hi]
            mode = choose_algorithm((hi - lo) * t.element_size(), self.world)
            self._call(mode, piece, piece, hi - lo, 0, scale)
        return True

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> bool:
        """``dist.reduce_scatter_tensor`` semantics: ``inp`` = W contiguous slices, ``out`` = this
        rank's reduced slice (it may be the input's own slice, in place). False: not eligible."""
        W = self.world
        if not (self.use["reduce_scatter"] and self.fits(inp) and out.is_contiguous() and out.dtype == inp.dtype and out.is_cuda
                and inp.numel() == W * out.numel() and out.data_ptr() % 16 == 0):
            return False
        ns = out.numel()
        es = inp.element_size()
        if (ns * es) % 16:
            return False
        scale = 1.0 / W if op == "avg" else 1.0
        fi, fo = inp.view(-1), out.view(-1)
        for lo, hi in _bands(ns, self.region // (W * es), 16 // es):
            self._call("reduce_scatter", fi[lo:], fo[lo:hi], hi - lo, ns, scale)
        return True

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> bool:
        """``dist.all_gather_into_tensor`` semantics (``inp`` may be ``out``'s own slice)."""
        W = self.world
        if not (self.use["all_gather"] and self.fits(out) and inp.is_contiguous() and inp.dtype == out.dtype and inp.is_cuda
                and out.numel() == W * inp.numel() and inp.data_ptr() % 16 == 0):
            return False
        ns = inp.numel()
        es = out.element_size()
        if (ns * es) % 16:
            return False
        fi, fo = inp.view(-1), out.view(-1)
        for lo, hi in _bands(ns, self.region // es, 16 // es):
            self._call("all_gather", fi[lo:hi], fo[lo:], hi - lo, ns, 1.0)
        return True

    def _async(self, fn, tensors, *args) -> Optional[_EventHandle]:
        dev = tensors[0].device
        if self._stream is None:
            from .streams import comm_stream
            self._stream = comm_stream(dev)
        cur = torch.cuda.current_stream(dev)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            ev0 = _timing_event(self._stream)
            ok = fn(*args)
            ev = torch.cuda.Event(enable_timing=ev0 is not None)
            ev.record(self._stream)
        if not ok:
            return None
        for t in tensors:
            t.record_stream(self._stream)
        return _EventHandle(ev, ev0)

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum") -> Optional[_EventHandle]:
        """The same on the engine's own stream, ordered after the current stream's work; returns
        a handle whose ``wait()`` makes the current stream wait (None: not eligible)."""
        if not (self.use["all_reduce"] and self.fits(t)):
            return None
        return self._async(self.all_reduce, [t], t, op)

    def reduce_scatter_async(self, out, inp, op: str = "sum") -> Optional[_EventHandle]:
        return self._async(self.reduce_scatter, [out, inp], out, inp, op)

    def all_gather_async(self, out, inp) -> Optional[_EventHandle]:
        return self._async(self.all_gather, [out, inp], out, inp)

    def _ag_range(self, flat: torch.Tensor, lo: int, hi: int, stride: int) -> bool:
        """All-gather elements [lo, hi) of every rank's slice of ``flat`` (slice r at r * stride,
        this rank's already in place), region-sized bands, one engine call each."""
        es = flat.element_size()
        mine = self.rank * stride
        for a, b in _bands(hi - lo, self.region // es, 16 // es):
            self._call("all_gather", flat[mine + lo + a:mine + lo + b], flat[lo + a:], b - a, stride, 1.0)
        return True

    def all_gather_pieces_async(self, flat: torch.Tensor, stride: int, ranges) -> Optional[List[_EventHandle]]:
        """``flat`` = W slices ``stride`` elements apart, this rank's in place; one engine call per
        element range of the slices (all peers' pieces at once, every link), issued in order on
        the engine stream; one handle per range (None: not eligible)."""
        if not (self.use["all_gather"] and self.fits(flat)):
            return None
        es = flat.element_size()
        if (stride * es) % 16 or any((lo * es) % 16 or (hi * es) % 16 for lo, hi in ranges):
            return None
        hs = []
        for lo, hi in ranges:
            h = self._async(self._ag_range, [flat], flat, lo, hi, stride)
            if h is None:
                return None
            hs.append(h)
        return hs

    def _rs_range(self, out: torch.Tensor, inp: torch.Tensor, lo: int, hi: int, stride: int) -> bool:
        es = inp.element_size()
        for a, b in _bands(hi - lo, self.region // (self.world * es), 16 // es):
            self._call("reduce_scatter", inp[lo + a:], out[lo + a:lo + b], b - a, stride, 1.0)
        return True

    def reduce_scatter_piece_async(self, out: torch.Tensor, inp: torch.Tensor, lo: int, hi: int,
                                   stride: int) -> Optional[_EventHandle]:
        """out[lo:hi] = sum over ranks of elements [lo, hi) of slice ``rank`` (``inp`` = W slices
        ``stride`` apart, ``out`` this rank's reduced slice, both flat), on the engine stream."""
        if not (self.use["reduce_scatter"] and self.fits(inp) and out.is_contiguous() and out.dtype == inp.dtype
                and out.data_ptr() % 16 == 0 and inp.numel() == self.world * stride):
            return None
        es = inp.element_size()
        if (stride * es) % 16 or (lo * es) % 16 or (hi * es) % 16:
            return None
        return self._async(self._rs_range, [out, inp], out, inp, lo, hi, stride)

    def error(self) -> int:
        return int(self.C.ar_read_error(self._sig)) if self._sig is not None else 0

    def check(self):
        """Raise if any call of this engine timed out waiting for a peer (synchronises)."""
        torch.cuda.synchronize()
        e = self.error()
        if e:
            raise RuntimeError(f"xGMI all-reduce: a peer did not arrive (error word {e}); outputs were NaN-filled")

    def close(self):
        """Collective over the group: unmap the peers' buffers, then free this rank's own."""
        self._close_ipc()
        self._sig = None
        self.active = False


def create_for_group(group, auto: bool = False, log=print, tune: bool = False, **kw) -> Optional[XgmiAllReduce]:
    """Collective over ``group``: an engine when xGMI collectives are wanted and possible, else
    None (with a warning when wanted but not set up). ``auto`` (the DDP gradient / parameter
    collectives): when neither ``SMDT_XGMI_ALLREDUCE`` nor the smddp backend decided, build the
    engine anyway, validate it, time each op against RCCL on this node and keep the ops it wins
    (rank 0 logs the bus bandwidths); None when it wins none. ``tune``: time and select per op even
    when the engine was asked for explicitly (the smddp process group)."""
    if not (dist.is_initialized() and torch.cuda.is_available()):
        return None
    explicit = wanted(group)
    if not explicit and not (auto and not explicitly_off()):
        return None
    if not rccl_backend(group):
        return None
    ws = dist.get_world_size(group)
    if ws not in (2, 4, 8):
        return None
    try:
        eng = XgmiAllReduce(group, **kw)
    except (RuntimeError, ValueError) as e:
        warnings.warn(f"xGMI all-reduce disabled for this group: {e}")
        return None
    if explicit and not tune:
        return eng
    try:
        res = eng.tune()
    except RuntimeError as e:
        warnings.warn(f"xGMI collectives disabled for this group: {e}")
        eng.close()
        return None
    TUNED[f"dp{ws}"] = {op: {"rccl_ms": round(a, 3), "xgmi_ms": round(b, 3), "xgmi": eng.use[op]}
                        for op, (a, b, _, _) in res.items()}
    if dist.get_rank() == dist.get_global_rank(group, 0) and log is not None:
        pretty = ", ".join(f"{op} rccl {a:.2f} ms ({c:.0f} GB/s) / xgmi {b:.2f} ms ({d:.0f} GB/s)"
                           for op, (a, b, c, d) in res.items())
        log(f"[smdt] DP group of {ws}: {pretty} -> xGMI kernel for {[k for k, v in eng.use.items() if v] or 'nothing'}")
    if not any(eng.use.values()):
        eng.close()
        return None
    return eng


class XgmiLoopback:
    """W virtual ranks in ONE process and ONE launch (tests and microbenchmarks on a single GPU):
    the exact kernel, barrier protocol and double-buffering, with plain device buffers instead of
    IPC mappings."""

    def __init__(self, world: int, region_bytes: int = 8 << 20, blocks: Optional[int] = None):
        assert world in (2, 4, 8)
        self.C = _ext.ext()
        self.world = world
        self.region = (int(region_bytes) + 4095) // 4096 * 4096
        self.blocks = blocks or max(1, min(DEFAULT_BLOCKS, 512 // world))
        self.data_ptrs = [self.C.ipc_malloc(4 * self.region, False) for _ in range(world)]
        self.sig_ptrs = [self.C.ipc_malloc(self.C.ar_signal_bytes(), True) for _ in range(world)]

    def all_reduce(self, x: torch.Tensor, two_shot: bool, scale: float = 1.0, out: Optional[torch.Tensor] = None):
        """x: [world, n] (row r = virtual rank r's input). Returns [world, n] (out may be x)."""
        out = torch.empty_like(x) if out is None else out
        self.C.xgmi_allreduce(x, out, self.data_ptrs, self.sig_ptrs, 0, self.world, self.region, two_shot,
                              self.blocks, scale)
        return out

    def reduce_scatter(self, x: torch.Tensor, scale: float = 1.0, out: Optional[torch.Tensor] = None):
        """x: [world, W * ns] (row r = virtual rank r's W slices). Returns [world, ns]: row r = the
        reduced slice r (``out`` may be a strided view into x, e.g. each rank's own slice)."""
        W = self.world
        ns = x.shape[1] // W
        out = torch.empty(W, ns, dtype=x.dtype, device=x.device) if out is None else out
        self.C.xgmi_collective(2, x, out, self.data_ptrs, self.sig_ptrs, 0, W, self.region, self.blocks, ns, ns, scale)
        return out

    def all_gather(self, x: torch.Tensor, out: Optional[torch.Tensor] = None):
        """x: [world, ns] (row r = virtual rank r's slice). Returns [world, W * ns]."""
        W = self.world
        ns = x.shape[1]
        out = torch.empty(W, W * ns, dtype=x.dtype, device=x.device) if out is None else out
        self.C.xgmi_collective(3, x, out, self.data_ptrs, self.sig_ptrs, 0, W, self.region, self.blocks, ns, ns, 1.0)
        return out

    def errors(self) -> List[int]:
        torch.cuda.synchronize()
        return [int(self.C.ar_read_error(s)) for s in self.sig_ptrs]

    def close(self):
        torch.cuda.synchronize()
        for p in self.data_ptrs + self.sig_ptrs:
            self.C.ipc_free(p)
        self.data_ptrs, self.sig_ptrs = [], []
