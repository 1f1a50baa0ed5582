"""Collective bandwidth vs message size: RCCL vs the xGMI IPC kernel (comm/xgmi.py).

    torchrun --nproc-per-node N --master-addr 127.0.0.1 benchmarks/bench_collectives.py [--max-mb 256]
    python benchmarks/bench_collectives.py --loopback 8          # one GPU: kernel only, no links

For every size from 48 KB to ``--max-mb`` (x4 steps) and every op — all-reduce, reduce-scatter,
all-gather (RCCL and xGMI) and all-to-all (RCCL) — prints one JSON line with the median time over
``--iters`` back-to-back calls and the bus bandwidth in the nccl-tests convention:

    all-reduce      busbw = bytes * 2 (W - 1) / W / t
    reduce-scatter  busbw = bytes * (W - 1) / W / t     (bytes = the full, unreduced tensor)
    all-gather      busbw = bytes * (W - 1) / W / t     (bytes = the gathered tensor)
    all-to-all      busbw = bytes * (W - 1) / W / t
    pair exchange   busbw = bytes / t     (every rank swaps ``bytes`` with its TP partner r ^ 1;
                                           RCCL p2p over the one direct link vs comm/relay.py)

That is the per-GPU link traffic rate: on an MI355X node each GPU has 7 xGMI links, so W = 8
collectives can approach 7 x the one-link rate while a W = 2 group is bound by its single link
(the reference's collectives are stock NCCL / SMDDP; the bucket sizes of
parallel/distributed.py and the TP degree are chosen from these curves).

``--loopback W`` times the xGMI kernel with W virtual ranks in one launch on ONE GPU (all
"peer" reads are local HBM reads): it measures the kernel's own cost (barriers, staging, the
reduction) — not link bandwidth — and is labelled ``"loopback": true``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from smdt_amd.comm import relay, xgmi  # noqa: E402

FACTOR = {"all_reduce": lambda w: 2.0 * (w - 1) / w, "reduce_scatter": lambda w: (w - 1) / w,
          "all_gather": lambda w: (w - 1) / w, "all_to_all": lambda w: (w - 1) / w,
          "pair_exchange": lambda w: 1.0}


def sizes(max_mb: float):
    s = 48 << 10
    out = []
    while s <= max_mb * (1 << 20):
        out.append(s)
        s *= 4
    return out


def timed(fn, iters: int, warmup: int, sync):
    for _ in range(warmup):
        fn()
    sync()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        fn()
        sync()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2]


def emit(rec):
    print(json.dumps(rec), flush=True)


def run_distributed(a):
    from smdt_amd.comm import init_distributed
    rank, local, world, backend = init_distributed("nccl")
    dev = torch.device("cuda", local)
    W = world

    def sync():
        torch.cuda.synchronize()
        dist.barrier()

    eng = None
    if W in (2, 4, 8):
        try:
            eng = xgmi.XgmiAllReduce(None, region_bytes=a.region_mb << 20)
        except (RuntimeError, ValueError) as e:
            if rank == 0:
                print(f"[bench_collectives] xGMI engine unavailable: {e}", flush=True)
    # TP-pair exchange (pairs r, r ^ 1): RCCL p2p vs the multi-path relay, every pair at once
    pairs = [dist.new_group([p, p + 1]) for p in range(0, W, 2)] if W % 2 == 0 else []
    rly = None
    if W in (4, 8):
        try:
            rly = relay.XgmiRelay(pairs[rank // 2])
        except (RuntimeError, ValueError) as e:
            if rank == 0:
                print(f"[bench_collectives] xGMI relay unavailable: {e}", flush=True)
    for nbytes in sizes(a.max_mb):
        n = nbytes // 2 // W * W                    # bf16 elements, divisible by W
        full = torch.randn(n, device=dev, dtype=torch.bfloat16)
        part = torch.empty(n // W, device=dev, dtype=torch.bfloat16)
        out_full = torch.empty_like(full)
        cases = [
            ("all_reduce", "rccl", lambda: dist.all_reduce(full)),
            ("reduce_scatter", "rccl", lambda: dist.reduce_scatter_tensor(part, full)),
            ("all_gather", "rccl", lambda: dist.all_gather_into_tensor(out_full, part)),
            ("all_to_all", "rccl", lambda: dist.all_to_all_single(out_full, full)),
        ]
        if eng is not None:
            cases += [("all_reduce", "xgmi", lambda: eng.all_reduce(full)),
                      ("reduce_scatter", "xgmi", lambda: eng.reduce_scatter(part, full)),
                      ("all_gather", "xgmi", lambda: eng.all_gather(out_full, part))]
        if pairs:
            pin, pout = torch.empty_like(full), torch.empty_like(full)
            cases.append(("pair_exchange", "rccl", lambda: dist.batch_isend_irecv(
                [dist.P2POp(dist.isend, full, rank ^ 1, pairs[rank // 2]),
                 dist.P2POp(dist.irecv, pin, rank ^ 1, pairs[rank // 2])])[-1].wait()))
            if rly is not None:
                cases.append(("pair_exchange", "relay", lambda: rly.exchange(full, pout)))
        for op, impl, fn in cases:
            t = timed(fn, a.iters, a.warmup, sync)
            if rank == 0:
                emit({"op": op, "impl": impl, "world": W, "bytes": n * 2, "ms": t * 1e3,
                      "busbw_GBps": n * 2 * FACTOR[op](W) / t / 1e9, "algbw_GBps": n * 2 / t / 1e9,
                      "loopback": False})
    if eng is not None:
        eng.check()
        eng.close()
    if rly is not None:
        rly.check()
        rly.close()
    dist.barrier()
    dist.destroy_process_group()


def run_loopback(a):
    W = a.loopback
    lb = xgmi.XgmiLoopback(W, region_bytes=a.region_mb << 20)
    sync = torch.cuda.synchronize
    try:
        for nbytes in sizes(min(a.max_mb, a.region_mb)):
            n = nbytes // 2 // W * W // 8 * 8
            x = torch.randn(W, n, device="cuda", dtype=torch.bfloat16)
            ns = n // W
            sl = torch.randn(W, ns, device="cuda", dtype=torch.bfloat16)
            cases = [("all_reduce", lambda: lb.all_reduce(x, xgmi.choose_algorithm(n * 2, W) == "two_shot")),
                     ("reduce_scatter", lambda: lb.reduce_scatter(x)),
                     ("all_gather", lambda: lb.all_gather(sl))]
            for op, fn in cases:
                t = timed(fn, a.iters, a.warmup, sync)
                emit({"op": op, "impl": "xgmi", "world": W, "bytes": n * 2, "ms": t * 1e3,
                      "busbw_GBps": n * 2 * FACTOR[op](W) / t / 1e9, "loopback": True,
                      "note": "W virtual ranks on one GPU: kernel cost only, no xGMI links"})
        assert lb.errors() == [0] * W, lb.errors()
    finally:
        lb.close()
    rl = relay.XgmiRelayLoopback(W, slot_bytes=a.region_mb << 20, sub=2)
    try:
        for nbytes in sizes(min(a.max_mb, W * a.region_mb // 2)):
            n = nbytes // 2 // 8 * 8
            x = torch.randn(W, n, device="cuda", dtype=torch.bfloat16)
            y = torch.empty_like(x)
            t = timed(lambda: rl.exchange(x, y), a.iters, a.warmup, sync)
            emit({"op": "pair_exchange", "impl": "relay", "world": W, "bytes": n * 2, "ms": t * 1e3,
                  "busbw_GBps": n * 2 / t / 1e9, "loopback": True,
                  "note": "W virtual ranks on one GPU: kernel cost only, no xGMI links"})
        assert rl.errors() == [0] * W, rl.errors()
    finally:
        rl.close()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--max-mb", type=float, default=256)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--region-mb", type=int, default=64)
    p.add_argument("--loopback", type=int, default=0, help="W virtual ranks on one GPU (2 / 4 / 8)")
    a = p.parse_args()
    if a.loopback:
        run_loopback(a)
    else:
        run_distributed(a)


if __name__ == "__main__":
    main()
