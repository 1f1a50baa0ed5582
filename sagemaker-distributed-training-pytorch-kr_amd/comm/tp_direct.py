"""Direct multi-link sequence-parallel exchanges for TP groups of 4 or 8 GPUs.

The sequence-parallel collective-matmul (parallel/tensor_parallel.ag_ring / rs_ring) moves one
[s/tp, b, h] chunk per ring step from each rank to its ring successor: on the all-to-all xGMI
mesh of an MI355X node that is ONE link per direction per rank, while the rank has tp - 1 links
into its TP group (3 at TP4). For GPT-3 6.7B at TP4 PP2 + SP (BASELINE config #5) a rank moves
~64 GB of SP traffic per step, ~1 s over one link against ~0.38 s of compute
(BENCHMARKS.md, benchmarks/predict_scaling.py).

``TpDirect`` replaces the ring, for TP groups larger than 2 (TP pairs have the relay engine,
comm/relay.py), by the single-launch all-gather / reduce-scatter of the xGMI engine
(comm/xgmi.XgmiAllReduce): every rank reads all of its peers' chunks at once, one per link, so
the exchange runs at (tp - 1) links per rank:

* all-gather (column-parallel forward, row-parallel backward): the gather starts on the engine's
  stream while the GEMM of the local chunk runs on the compute stream, then the peers' chunks;
* reduce-scatter (row-parallel forward, column-parallel backward): the partial products of all
  chunks, then one engine reduce-scatter, beside which the backward runs its queued weight-gradient
  GEMMs (the ring's ``before_last_wait``).

It is built at ``initialize_model_parallel`` for TP groups of 4 / 8 on a node whose backend is
RCCL (collective over the TP group), checked bit-exactly against RCCL by the engine's own
validation, and KEPT ONLY WHEN a timed all-gather at a representative chunk size beats the ring on
every rank (``SMDT_TP_DIRECT=1`` / ``0`` forces it on / off). ``TpDirect.for_test(group)`` builds
it without validation or timing over a Gloo group (multi-process tests sharing one GPU).
"""
from __future__ import annotations

import os
import time
from typing import Callable, Optional

import torch
import torch.distributed as dist

TUNED: dict = {}
# Row pieces per direct exchange (SMDT_TP_DIRECT_PIECES): piece j's GEMMs start when piece j has
# landed (all-gather) / piece j's reduce-scatter runs beside piece j + 1's GEMMs. 1 = whole chunks,
# the peers' rows in one GEMM per contiguous run and every partial in one GEMM: measured fastest on
# the emulated GPT-3 tp4 stage under the paced engine stand-in (532 vs 590 ms at 2 pieces, 694 at
# 4: the per-piece GEMMs of M = 1,024 rows fill a quarter of the chip; profiles/r6_direct/).
PIECES = max(1, int(os.environ.get("SMDT_TP_DIRECT_PIECES", "1")))


class TpDirect:
    def __init__(self, engine, group, world: Optional[int] = None, rank: Optional[int] = None):
        self.eng = engine
        self.group = group
        self.world = dist.get_world_size(group) if world is None else int(world)
        self.rank = dist.get_rank(group) if rank is None else int(rank)
        self.calls = 0
        self.pieces_issued = 0

    @classmethod
    def for_test(cls, group, region_bytes: int = 8 << 20) -> "TpDirect":
        from .xgmi import XgmiAllReduce
        return cls(XgmiAllReduce(group, region_bytes=region_bytes, blocks=32, validate=False), group)

    @property
    def active(self) -> bool:
        return self.eng is not None and self.eng.active

    def fits(self, t: torch.Tensor) -> bool:
        """Whether the engine takes a tensor shaped like ``t``. World-uniform facts only (TP ranks
        exchange equal shapes and dtypes; ``active`` changes only by a world-agreed fallback):
        a rank that ran the ring while a peer ran the engine would deadlock the group. Address
        alignment is not asked here: the engine only ever sees the freshly allocated (512-byte
        aligned) gather / staging buffers below, never the caller's views."""
        nb = t.numel() * t.element_size()
        return self.active and t.is_cuda and t.dtype in (torch.bfloat16, torch.float16, torch.float32) \
            and nb > 0 and nb % 16 == 0

    def _pieces(self, n: int, row_bytes: int):
        """Row pieces [a, b) of an n-row chunk: ``PIECES`` equal ones when n divides and every
        piece starts on a 16-byte boundary, else one. World-uniform (shapes only)."""
        k = max(1, min(PIECES, n))
        while k > 1 and n % k:
            k -= 1
        if row_bytes % 16:
            k = 1
        p = n // k
        return [(j * p, (j + 1) * p) for j in range(k)]

    def all_gather(self, x: torch.Tensor, chunk_fn: Optional[Callable] = None,
                   before_last_wait: Optional[Callable] = None) -> Optional[torch.Tensor]:
        """``ag_ring`` semantics: returns the gathered [ws * n, ...] tensor after calling
        ``chunk_fn(lo, rows)`` on every gathered row range. The gather runs as row pieces, each
        piece ONE engine call that reads that piece of every peer's chunk at once (all of the
        group's links); the local chunk's GEMM runs beside the first piece, and the peers' rows
        of piece j as soon as piece j has landed (its event), beside piece j + 1's transfer.
        None: not applicable (the caller runs the ring)."""
        x = x.contiguous()
        if not (self.fits(x) and self.eng.use["all_gather"]):
            return None
        ws, r, n = self.world, self.rank, x.shape[0]
        total = x.new_empty((n * ws,) + tuple(x.shape[1:]))
        total[r * n:(r + 1) * n].copy_(x)
        row = x[0].numel() if n else 0
        pieces = self._pieces(n, row * x.element_size())
        hs = self.eng.all_gather_pieces_async(total.view(-1), n * row, [(a * row, b * row) for a, b in pieces])
        if hs is None:     # cannot happen for a tensor fits() took: refuse loudly instead of mixing paths
            raise RuntimeError("TpDirect.all_gather: the xGMI engine refused an exchange fits() accepted")
        self.calls += 1
        self.pieces_issued += len(pieces)
        if chunk_fn is not None:
            chunk_fn(r * n, x)                   # beside the first piece
        from ..parallel.tensor_parallel import _wait_works, fill_exchange_wait
        for j, (a, b) in enumerate(pieces):
            if j == len(pieces) - 1 and before_last_wait is not None:
                before_last_wait()
            fill_exchange_wait()      # queued W GEMMs beside the piece in flight (SMDT_W_FILL)
            _wait_works([hs[j]], self.group)       # (counted as TP exchange wait by comm/stats)
            if chunk_fn is None:
                continue
            if len(pieces) == 1:
                # whole chunks: the peers' rows are (at most) two contiguous runs, one GEMM each
                for c0, c1 in ((r + 1, ws), (0, r)):
                    if c1 > c0:
                        chunk_fn(c0 * n, total[c0 * n:c1 * n])
                continue
            for d in range(1, ws):
                c = (r + d) % ws
                chunk_fn(c * n + a, total[c * n + a:c * n + b])
        return total

    def start_all_gather(self, x: torch.Tensor):
        """Issue the whole-chunk gather of ``x`` now and return (gathered buffer, handles) without
        waiting (the sub-batch interleave, ``tensor_parallel.ag_start``: the other batch half's
        phase runs beside the transfer); None when the engine does not take ``x``."""
        x = x.contiguous()
        if not (self.fits(x) and self.eng.use["all_gather"]):
            return None
        ws, r, n = self.world, self.rank, x.shape[0]
        total = x.new_empty((n * ws,) + tuple(x.shape[1:]))
        total[r * n:(r + 1) * n].copy_(x)
        row = x[0].numel() if n else 0
        hs = self.eng.all_gather_pieces_async(total.view(-1), n * row, [(0, n * row)])
        if hs is None:
            raise RuntimeError("TpDirect.start_all_gather: the xGMI engine refused an exchange fits() accepted")
        self.calls += 1
        self.pieces_issued += 1
        return total, hs

    def start_reduce_scatter(self, full: torch.Tensor):
        """Issue the reduce-scatter of the complete [ws * n, ...] partials ``full`` now and return
        (this rank's output chunk, handles) without waiting (sub-batch interleave); None when the
        engine does not take ``full``."""
        full = full.contiguous()
        if not (self.fits(full) and self.eng.use["reduce_scatter"]):
            return None
        n = full.shape[0] // self.world
        row = full[0].numel() if n else 0
        out = full.new_empty((n,) + tuple(full.shape[1:]))
        h = self.eng.reduce_scatter_piece_async(out.view(-1), full.view(-1), 0, n * row, n * row)
        if h is None:
            raise RuntimeError("TpDirect.start_reduce_scatter: the xGMI engine refused an exchange fits() accepted")
        self.calls += 1
        self.pieces_issued += 1
        return out, [h]

    def reduce_scatter(self, partial_fn: Callable, full_shape, ref: torch.Tensor,
                       before_last_wait: Optional[Callable] = None) -> torch.Tensor:
        """``rs_ring`` semantics: ``partial_fn(lo, rows, out)`` writes rows [lo, lo + rows) of the
        [ws * n, ...] tensor being reduced (``full_shape``, ``ref``'s dtype / device) into ``out``;
        returns this rank's reduced chunk. Push-style in row pieces: piece j's partials of every
        chunk go straight into the engine's input buffer (no staging copy of whole partials), then
        ONE engine reduce-scatter of that piece over all links runs on the engine stream while the
        GEMMs of piece j + 1 run. RCCL's reduce-scatter when the engine cannot take the buffer."""
        ws, r = self.world, self.rank
        full_shape = tuple(full_shape)
        n = full_shape[0] // ws
        buf = torch.empty(full_shape, dtype=ref.dtype, device=ref.device)
        out = buf.new_empty((n,) + full_shape[1:])
        row = buf[0].numel() if n else 0
        if not (self.fits(buf) and self.eng.use["reduce_scatter"]):
            for c in range(ws):
                partial_fn(c * n, n, buf[c * n:(c + 1) * n])
            w = dist.reduce_scatter_tensor(out, buf, group=self.group, async_op=True)
            if before_last_wait is not None:
                before_last_wait()
            w.wait()
            return out
        pieces = self._pieces(n, row * buf.element_size())
        hs = []
        for a, b in pieces:
            if len(pieces) == 1:                 # whole chunks: every chunk's partial in ONE GEMM
                partial_fn(0, ws * n, buf)
                hs.append(self.eng.reduce_scatter_piece_async(out.view(-1), buf.view(-1), 0, n * row, n * row))
                if hs[-1] is None:
                    raise RuntimeError("TpDirect.reduce_scatter: the xGMI engine refused an exchange fits() accepted")
                continue
            for d in range(1, ws + 1):           # the peers' rows first, this rank's own last
                c = (r + d) % ws
                partial_fn(c * n + a, b - a, buf[c * n + a:c * n + b])
            h = self.eng.reduce_scatter_piece_async(out.view(-1), buf.view(-1), a * row, b * row, n * row)
            if h is None:
                raise RuntimeError("TpDirect.reduce_scatter: the xGMI engine refused an exchange fits() accepted")
            hs.append(h)
        self.calls += 1
        self.pieces_issued += len(pieces)
        if before_last_wait is not None:
            before_last_wait()
        from ..parallel.tensor_parallel import _wait_works, fill_exchange_wait
        fill_exchange_wait()          # queued W GEMMs beside the last pieces in flight (SMDT_W_FILL)
        _wait_works(hs, self.group)
        return out


def create(group) -> Optional[TpDirect]:
    """Collective over the TP ``group`` (4 or 8 ranks on one node): the engine when it is wanted
    and measured faster than the p2p ring, else None."""
    env = os.environ.get("SMDT_TP_DIRECT")
    if env == "0" or not (dist.is_initialized() and torch.cuda.is_available()):
        return None
    from . import xgmi
    ws = dist.get_world_size(group)
    if ws not in (4, 8) or not xgmi.rccl_backend(group):
        return None
    try:
        eng = xgmi.XgmiAllReduce(group)
    except (RuntimeError, ValueError) as e:
        import warnings
        warnings.warn(f"direct TP exchanges disabled: {e}")
        return None
    td = TpDirect(eng, group)
    if env == "1":
        return td
    # time the ring against the engine: one [s/tp, b, h]-sized all-gather (8 MB per rank)
    from ..parallel.tensor_parallel import ag_ring
    dev = torch.device("cuda", torch.cuda.current_device())
    x = torch.randn(4096, 1024, device=dev, dtype=torch.bfloat16)
    ts = []
    for fn in (lambda: ag_ring(x, group, _skip_direct=True), lambda: td.all_gather(x)):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = torch.tensor([(time.perf_counter() - t0) / 5], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        ts.append(float(t.item()))
    TUNED[f"tp{ws}"] = {"ring_ms": round(ts[0] * 1e3, 3), "direct_ms": round(ts[1] * 1e3, 3),
                        "direct": ts[1] < ts[0]}
    if ts[1] < ts[0]:
        return td
    eng.close()
    return None
