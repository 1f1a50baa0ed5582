#!/usr/bin/env python3
"""Isolates the round-3 N = 4 rehearsal stall (profiles/r3_rehearse/): N processes on ONE GPU, a
Gloo process group, and the DP bucket pattern of bench.py's ZeRO-1 step — ``--buckets``
asynchronous ``reduce_scatter_tensor`` calls on CUDA tensors issued back to back, in the same
order on every rank, then waited in order — with no model, no DDP and no other collective.

    torchrun --nproc-per-node 4 benchmarks/gloo_cuda_probe.py --buckets 75 --mb 16

Prints one JSON line per rank: whether every reduce-scatter completed within ``--limit`` seconds
and the result was right (each rank contributes rank + 1, so every output element is
sum(1..N)). A stall here, with the identical issue order traced on every rank, points at Gloo's
CUDA-tensor collectives rather than at the framework's bucket order.
"""
import argparse
import json
import os
import threading
import time

import torch
import torch.distributed as dist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", type=int, default=75)
    ap.add_argument("--mb", type=float, default=16.0)
    ap.add_argument("--limit", type=float, default=60.0)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    dev = torch.device(a.device, 0) if a.device == "cuda" else torch.device("cpu")
    n = int(a.mb * 2 ** 20 / 4) // w * w
    bufs = [torch.full((n,), float(r + 1), device=dev) for _ in range(a.buckets)]
    outs = [torch.empty(n // w, device=dev) for _ in range(a.buckets)]
    done = {"k": 0}
    res = {"rank": r, "world": w, "buckets": a.buckets, "MB": a.mb, "device": str(dev)}

    def watchdog():
        t0 = time.time()
        while done["k"] < a.buckets and time.time() - t0 < a.limit:
            time.sleep(0.5)
        if done["k"] < a.buckets:
            print(json.dumps({**res, "completed": done["k"], "stalled": True}), flush=True)
            os._exit(3)
    threading.Thread(target=watchdog, daemon=True).start()
    t0 = time.time()
    works = [dist.reduce_scatter_tensor(outs[i], bufs[i], async_op=True) for i in range(a.buckets)]
    for wk in works:
        wk.wait()
        done["k"] += 1
    if dev.type == "cuda":
        torch.cuda.synchronize()
    want = float(w * (w + 1) // 2)
    ok = all(bool((o == want).all()) for o in outs)
    print(json.dumps({**res, "completed": done["k"], "stalled": False, "correct": ok,
                      "seconds": round(time.time() - t0, 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
