"""Multi-path exchange for tensor-parallel pairs over every xGMI link of an MI355X node.

A TP=2 layout (the BASELINE's TP2 x PP2 x DP2) moves each sequence-parallel chunk between the
two GPUs of a pair once per ring step (``parallel/tensor_parallel.ag_ring`` / ``rs_ring``: 8
exchanges of 16 MB per layer and micro-batch for GPT-2 345M at micro-batch 16). xGMI is point-to-
point: the pair shares ONE link (~64-77 GB/s per direction) while each GPU's 6 other links idle,
so RCCL's p2p send/recv moves a layer's activations slower than the MFMA cores consume them.

``XgmiRelay`` cuts every message into W parts: 2 go directly into the partner's staging buffer,
W - 2 are staged in the other GPUs' buffers and pulled from there by the partner
(``csrc/kernels/xgmi_relay.hip``; the relays run no code). With all pairs of a node exchanging at
once every directed link carries 2/W of a message — ~4x the one-link rate on 8 GPUs.

Construction is collective over the WORLD (every GPU of the node is a waypoint). It is only kept
when it (1) reproduces RCCL's exchange exactly and (2) is measured faster than RCCL's p2p
exchange at the message sizes it will carry — the decision is made at run time from a timing on
the real links, agreed by all ranks, and logged. ``SMDT_TP_RELAY=0`` turns it off, ``=1`` skips
the speed test (correctness is always checked).

Timeouts: every wait of the relay kernel gives up after ``spin_limit`` polls of an uncached word
(default 2^22, i.e. seconds; ``set_spin_limit``), NaN-fills and sets a sticky error word. That
bound is far above any collective, but a host stall of seconds on one partner (a slow filesystem,
a rank-local evaluation) can reach it; the health monitor (comm/health.py) then agrees on the error
over the world at the next step boundary and switches every engine off — the run continues on RCCL
p2p, the step that saw NaN activations is skipped by found-inf. Nothing stays poisoned.

The reference's TP collectives are stock NCCL; there is nothing to port.
"""
from __future__ import annotations

import os
import time
import warnings
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import _ext
from . import health
from .xgmi import IpcEngine, _EventHandle, _timing_event

DEFAULT_SLOT_BYTES = 8 << 20      # per (flow, parity): parts of up to 4 MB -> 32 MB per call on 8 GPUs
DEFAULT_SUB = 4                   # blocks per part and direction (2 x W x 4 = 64 blocks on 8 GPUs)
_ENGINES: Dict[int, "XgmiRelay"] = {}
TUNED: Dict[str, dict] = {}  # run-time RCCL-vs-relay timings (bench JSON)


def mode() -> str:
    """'off' / 'auto' (validated + timed against RCCL) / 'on' (validated only)."""
    v = os.environ.get("SMDT_TP_RELAY", "auto").lower()
    return {"0": "off", "off": "off", "1": "on", "on": "on"}.get(v, "auto")


def engine_for(group) -> Optional["XgmiRelay"]:
    return _ENGINES.get(id(group)) if group is not None else None


def eligible(send: torch.Tensor, recv: torch.Tensor) -> bool:
    nbytes = send.numel() * send.element_size()
    return (send.is_cuda and send.is_contiguous() and recv.is_contiguous() and send.dtype == recv.dtype
            and send.numel() == recv.numel() and send.dtype in (torch.float32, torch.bfloat16, torch.float16)
            and nbytes > 0 and nbytes % 16 == 0 and send.data_ptr() % 16 == 0 and recv.data_ptr() % 16 == 0)


class XgmiRelay(IpcEngine):
    """Pairwise exchange engine for the size-2 ``pair_group`` of every rank (collective over WORLD)."""

    def __init__(self, pair_group, slot_bytes: int = DEFAULT_SLOT_BYTES, sub: int = DEFAULT_SUB,
                 validate: bool = True):
        self.group = pair_group
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        if self.world not in (2, 4, 8):
            raise ValueError(f"xGMI relay supports 2, 4 or 8 ranks, not {self.world}")
        if dist.get_world_size(pair_group) != 2:
            raise ValueError("xGMI relay exchanges within groups of 2 ranks")
        self.slot = (int(slot_bytes) + 4095) // 4096 * 4096
        self.sub = int(sub)
        self.epoch = 0
        self.min_bytes = 0
        self.calls = 0
        self._stream = None
        self._sig = None
        self.active = False
        self.partner = [r for r in dist.get_process_group_ranks(pair_group) if r != self.rank][0]
        partners = [None] * self.world
        dist.all_gather_object(partners, self.partner)
        self.partners = [int(p) for p in partners]
        if any(self.partners[p] != r for r, p in enumerate(self.partners)):
            raise RuntimeError(f"xGMI relay: pair groups are not symmetric: {self.partners}")
        self.stage_ptrs, self.sig_ptrs = self._setup_ipc(None, [(self.world * 2 * self.slot, False),
                                                                (_ext.ext().relay_signal_bytes(), True)])
        self._sig = self.sig_ptrs[self.rank]
        self.active = True
        if validate and not self._validate():
            self.close()
            raise RuntimeError("xGMI relay failed its validation against RCCL p2p")
        health.register(self)

    _WORD_OFFSET = "relay_word_offset"
    # [s / tp, mbs, h] bf16 = 512 x 16 x 1024 x 2 B at the N = 8 bench layout (tp2, mbs 16)
    RING_CHUNK_BYTES = 16 << 20

    # ------------------------------------------------------------------ helpers
    def _rccl_exchange(self, send, recv):
        """The reference exchange: RCCL p2p (gloo test groups: through host copies)."""
        host = dist.get_backend(self.group) == "gloo"
        s, r = (send.cpu(), torch.empty(recv.shape, dtype=recv.dtype)) if host else (send, recv)
        works = dist.batch_isend_irecv([dist.P2POp(dist.isend, s, self.partner, self.group),
                                        dist.P2POp(dist.irecv, r, self.partner, self.group)])
        for w in works:
            w.wait()
        if host:
            recv.copy_(r)

    def _validate(self) -> bool:
        """Exact check against RCCL p2p on rank-tagged data: three calls (both slot parities and
        the slot-reuse wait), an odd size that leaves parts short, bf16 and fp32, and a message
        larger than one call."""
        dev = torch.device("cuda", torch.cuda.current_device())
        good = True
        big = self.world * self.slot // 2 // 4 + 4096  # fp32 elements: more than one call
        ring = self.RING_CHUNK_BYTES // 2              # bf16: one SP ring chunk of the N = 8 bench
        for n, dt, reps in ((4096, torch.float32, 3), (1000 * 8 + 8, torch.bfloat16, 3), (big, torch.float32, 3),
                            (ring, torch.bfloat16, 1)):
            for rep in range(reps):
                x = ((torch.arange(n, device=dev, dtype=torch.float32) % 251) + 1000.0 * self.rank + rep).to(dt)
                ref = torch.empty_like(x)
                self._rccl_exchange(x, ref)
                got = torch.empty_like(x)
                self.exchange(x, got)
                good &= bool(torch.equal(got, ref))
        torch.cuda.synchronize()
        good &= self.error() == 0
        return self._agree(good)

    def tune(self, sizes=(1 << 20, 4 << 20, 16 << 20), iters: int = 10) -> Dict[int, tuple]:
        """Time RCCL p2p vs the relay with every pair of the node exchanging at once (the training
        pattern) and keep the relay for messages >= the smallest size where it wins on every rank
        (disabled when it never wins). Returns {bytes: (rccl_ms, relay_ms)} (max over ranks)."""
        dev = torch.device("cuda", torch.cuda.current_device())
        res = {}
        wins = []
        for nb in sizes:
            x = torch.randn(nb // 2, device=dev, dtype=torch.bfloat16)
            y = torch.empty_like(x)
            ts = []
            for fn in (lambda: self._rccl_exchange(x, y), lambda: self.exchange(x, y)):
                for _ in range(3):
                    fn()
                torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(iters):
                    fn()
                torch.cuda.synchronize()
                host = dist.get_backend() == "gloo"
                t = torch.tensor([(time.perf_counter() - t0) / iters * 1e3], device="cpu" if host else dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                ts.append(float(t.item()))
            res[nb] = tuple(ts)
            wins.append(ts[1] < ts[0])
        self.min_bytes = next((nb for nb, w in zip(sizes, wins) if w and all(wins[sizes.index(nb):])), None)
        if self.min_bytes is None:
            self.active = False
        return res

    def tune_sub(self, candidates=(1, 2, 4), nbytes: int = 16 << 20, iters: int = 10, tol: float = 1.05) -> dict:
        """Pick the blocks per part and direction (``sub``): the kernel keeps 2 x world x sub
        workgroups resident for a whole exchange, one CU each, which the rank's chunk GEMMs then do
        without (tensor_parallel.gemm_tn_blocks; 16 vs 64 held CUs, profiles/r6_mix/). Times every
        candidate with all pairs exchanging at once (max over ranks, so every rank decides alike)
        and keeps the smallest within ``tol`` of the fastest. Returns {sub: ms}."""
        dev = torch.device("cuda", torch.cuda.current_device())
        x = torch.randn(nbytes // 2, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        keep = self.sub
        res = {}
        host = dist.get_backend() == "gloo"
        for sub in candidates:
            self._set_sub(int(sub))
            for _ in range(3):
                self.exchange(x, y)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                self.exchange(x, y)
            torch.cuda.synchronize()
            t = torch.tensor([(time.perf_counter() - t0) / iters * 1e3], device="cpu" if host else dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            res[int(sub)] = float(t.item())
        best = min(res.values())
        self._set_sub(min(sb for sb, t in res.items() if t <= tol * best) if res else keep)
        return res

    def _set_sub(self, sub: int):
        """Change the blocks per part between exchanges: the (part, block) -> sub-range map
        changes, so every rank drains, the flags and device epochs are zeroed (partners stay
        equal: both restart at epoch 1) and every rank resumes together. Collective over WORLD."""
        if sub == self.sub:
            return
        torch.cuda.synchronize()
        dist.barrier()
        self.C.relay_reset(self.sig_ptrs[self.rank])
        torch.cuda.synchronize()
        dist.barrier()
        self.sub = int(sub)

    # ------------------------------------------------------------------ API
    def cu_blocks(self) -> int:
        """Workgroups the relay kernel keeps resident during an exchange (one CU each)."""
        return 2 * self.world * self.sub

    def fits(self, send, recv) -> bool:
        return (self.active and eligible(send, recv)
                and send.numel() * send.element_size() >= (self.min_bytes or 0))

    def exchange(self, send: torch.Tensor, recv: torch.Tensor) -> bool:
        """recv (this rank) <- send (partner), both flat-contiguous, on the current stream. Calls
        must be issued in the same order and sizes on both partners (they are: ring steps)."""
        if not (self.active and eligible(send, recv)):
            return False
        es = send.element_size()
        per = self.world * (self.slot // 32) * 16 // es      # elements per call (2 parts per slot)
        fs, fr = send.view(-1), recv.view(-1)
        n = fs.numel()
        step = max(16 // es, per // (16 // es) * (16 // es))
        # device epochs: call i of this exchange runs at (this rank's device call counter) + i, and
        # one bump after the calls advances the counter — identical on both partners, and correct
        # when a HIP graph replays a captured exchange (no host value is baked into the launches)
        i = 0
        for lo in range(0, n, step):
            hi = min(n, lo + step)
            i += 1
            self.C.xgmi_relay(fs[lo:hi], fr[lo:hi], self.stage_ptrs, self.sig_ptrs, self.partners, self.rank, 1,
                              self.slot, self.sub, i, True)
        self.C.relay_epoch_bump(self.sig_ptrs, self.rank, 1, i)
        self.epoch += i
        self.calls += 1
        return True

    def exchange_async(self, send: torch.Tensor, recv: torch.Tensor) -> Optional[_EventHandle]:
        """The same on the engine's side stream after the current stream's work; ``wait()`` on the
        handle makes the current stream wait. None: not taken (use RCCL)."""
        if not self.fits(send, recv):
            return None
        dev = send.device
        if self._stream is None:
            from .streams import comm_stream
            self._stream = comm_stream(dev)
        cur = torch.cuda.current_stream(dev)
        self._stream.wait_stream(cur)
        with torch.cuda.stream(self._stream):
            ev0 = _timing_event(self._stream)
            self.exchange(send, recv)
            ev = torch.cuda.Event(enable_timing=ev0 is not None)
            ev.record(self._stream)
        send.record_stream(self._stream)
        recv.record_stream(self._stream)
        return _EventHandle(ev, ev0)

    def error(self) -> int:
        return int(self.C.relay_read_error(self._sig)) if self._sig is not None else 0

    def check(self):
        torch.cuda.synchronize()
        e = self.error()
        if e:
            raise RuntimeError(f"xGMI relay: the partner did not arrive (error word {e}); outputs were NaN-filled")

    def close(self):
        """Collective over WORLD: unmap the peers' buffers, then free this rank's own."""
        self._close_ipc()
        self._sig = None
        self.active = False
        for k, v in list(_ENGINES.items()):
            if v is self:
                del _ENGINES[k]


def check_all():
    """Raise if an ACTIVE relay engine's partner timed out (synchronises; call at logging points,
    not per step). An engine the health monitor already switched off (comm/health.py) is skipped:
    its error was handled by falling back to RCCL."""
    for eng in list(_ENGINES.values()):
        if eng.active:
            eng.check()


def create_for_pairs(pair_group, log=print) -> Optional[XgmiRelay]:
    """Collective over WORLD: build, validate and (mode 'auto') time the relay for this rank's
    TP pair; registered for ``pair_group`` when kept. None when off / not applicable / slower."""
    m = mode()
    if m == "off" or not (dist.is_initialized() and torch.cuda.is_available()):
        return None
    try:
        if dist.get_backend() not in ("nccl", "smddp") or dist.get_world_size() not in (4, 8):
            return None
        eng = XgmiRelay(pair_group)
    except (RuntimeError, ValueError) as e:
        warnings.warn(f"xGMI relay disabled: {e}")
        return None
    if m == "auto":
        res = eng.tune()
        TUNED["tp_pair"] = {f"{nb >> 20}MB": {"rccl_ms": round(a, 3), "relay_ms": round(b, 3)}
                            for nb, (a, b) in res.items()}
        TUNED["tp_pair"]["relay_min_bytes"] = eng.min_bytes if eng.active else None
        if eng.active:
            subs = eng.tune_sub()
            TUNED["tp_pair"]["relay_sub_ms"] = {str(k): round(v, 3) for k, v in subs.items()}
            TUNED["tp_pair"]["relay_sub"] = eng.sub
            TUNED["tp_pair"]["relay_cu_blocks"] = eng.cu_blocks()
        if dist.get_rank() == 0 and log is not None:
            pretty = ", ".join(f"{nb >> 20} MB: rccl {a:.3f} ms / relay {b:.3f} ms" for nb, (a, b) in res.items())
            log(f"[smdt] TP-pair exchange over all xGMI links: {pretty} -> "
                + (f"relay for messages >= {eng.min_bytes >> 10} KB" if eng.active else "RCCL kept"))
        if not eng.active:
            eng.close()
            return None
    _ENGINES[id(pair_group)] = eng
    return eng


class XgmiRelayLoopback:
    """W virtual ranks in ONE launch on one GPU (pairs (0,1), (2,3), ...): the exact kernel and
    protocol with plain device buffers (tests / kernel-cost microbenchmarks)."""

    def __init__(self, world: int, slot_bytes: int = 1 << 20, sub: int = 2):
        assert world in (2, 4, 8)
        self.C = _ext.ext()
        self.world = world
        self.slot = (int(slot_bytes) + 4095) // 4096 * 4096
        self.sub = sub
        self.epoch = 0
        self.partners = [r ^ 1 for r in range(world)]
        self.stage_ptrs = [self.C.ipc_malloc(world * 2 * self.slot, False) for _ in range(world)]
        self.sig_ptrs = [self.C.ipc_malloc(self.C.relay_signal_bytes(), True) for _ in range(world)]

    def exchange(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, epoch: Optional[int] = None,
                 device_epoch: bool = False):
        """x: [world, n] (row r = virtual rank r's message). Returns [world, n]: row r = row r^1 of x.
        ``device_epoch``: the engine's mode — the epoch comes from each virtual rank's device call
        counter, advanced by one bump after the call (graph-replayable)."""
        out = torch.empty_like(x) if out is None else out
        if device_epoch:
            self.C.xgmi_relay(x, out, self.stage_ptrs, self.sig_ptrs, self.partners, 0, self.world, self.slot,
                              self.sub, 1, True)
            self.C.relay_epoch_bump(self.sig_ptrs, 0, self.world, 1)
            return out
        self.epoch = self.epoch + 1 if epoch is None else epoch
        self.C.xgmi_relay(x, out, self.stage_ptrs, self.sig_ptrs, self.partners, 0, self.world, self.slot, self.sub,
                          self.epoch)
        return out

    def errors(self) -> List[int]:
        torch.cuda.synchronize()
        return [int(self.C.relay_read_error(s)) for s in self.sig_ptrs]

    def close(self):
        torch.cuda.synchronize()
        for p in self.stage_ptrs + self.sig_ptrs:
            self.C.ipc_free(p)
        self.stage_ptrs, self.sig_ptrs = [], []
