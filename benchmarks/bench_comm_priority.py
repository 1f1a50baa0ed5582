"""Does a communication kernel wait behind a chip-filling GEMM?  

One MI355X. A queue of bf16 GEMMs at a ring-chunk-like shape fills every CU on the compute
stream; while it runs, an 8-virtual-rank xGMI loopback collective (comm/xgmi.XgmiLoopback: the
engine's kernel, barrier protocol and double buffering in one launch — its blocks spin on each
other, so it is exactly the kind of kernel that stalls when only part of it is dispatched) is
issued on a side stream created at normal and at high priority (comm/streams.comm_stream). We
report the side stream's issue-to-completion latency, its latency on an idle GPU, and the GEMM
queue's time, median over rounds, both priorities interleaved in one process.

    python benchmarks/bench_comm_priority.py [--rounds 15] [--gemms 12] [--mb 8]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=15)
    p.add_argument("--gemms", type=int, default=12)
    p.add_argument("--mb", type=int, default=8, help="per-virtual-rank all-gather slice, MB")
    p.add_argument("--m", type=int, default=16384)
    p.add_argument("--n", type=int, default=3072)
    p.add_argument("--k", type=int, default=1024)
    p.add_argument("--delay-gemms", type=int, default=2, help="GEMMs queued before the collective")
    a = p.parse_args()
    from smdt_amd.comm.xgmi import XgmiLoopback
    dev = torch.device("cuda", 0)
    lo, hi = torch.cuda.Stream.priority_range()
    W = 8
    ns = a.mb * (1 << 20) // 2
    lb = XgmiLoopback(W, region_bytes=max(8 << 20, a.mb << 20))
    x = torch.randn(W, ns, device=dev, dtype=torch.bfloat16)
    out = torch.empty(W, W * ns, device=dev, dtype=torch.bfloat16)
    A = torch.randn(a.m, a.k, device=dev, dtype=torch.bfloat16)
    B = torch.randn(a.n, a.k, device=dev, dtype=torch.bfloat16)
    C = torch.empty(a.m, a.n, device=dev, dtype=torch.bfloat16)
    streams = {"normal": torch.cuda.Stream(device=dev, priority=lo), "high": torch.cuda.Stream(device=dev, priority=hi)}
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

    def idle(s):
        e0, e1 = ev(), ev()
        with torch.cuda.stream(s):
            e0.record()
            lb.all_gather(x, out)
            e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    def contended(s):
        cur = torch.cuda.current_stream()
        g0, g1, e0, e1 = ev(), ev(), ev(), ev()
        g0.record(cur)
        for i in range(a.gemms):
            torch.matmul(A, B.t(), out=C)
            if i == a.delay_gemms - 1:
                # the collective's dependency is met here: it is issued while the queue runs
                s.wait_stream(cur)
                with torch.cuda.stream(s):
                    e0.record()
                    lb.all_gather(x, out)
                    e1.record()
        g1.record(cur)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1), g0.elapsed_time(g1)

    for s in streams.values():        # warm up kernels, GEMM algorithm
        idle(s)
        contended(s)
    res = {k: {"idle": [], "lat": [], "gemm": []} for k in streams}
    for _ in range(a.rounds):
        for k, s in streams.items():
            res[k]["idle"].append(idle(s))
            lat, g = contended(s)
            res[k]["lat"].append(lat)
            res[k]["gemm"].append(g)
    errs = lb.errors()
    lb.close()
    gemm_ms = statistics.median(res["normal"]["gemm"]) / a.gemms
    out_rec = {"metric": "comm kernel issue-to-completion latency under a chip-filling GEMM queue",
               "unit": "ms", "priority_range": [lo, hi], "collective": f"xgmi loopback all-gather W=8, {a.mb} MB/rank",
               "gemm": f"{a.m}x{a.n}x{a.k} bf16 x{a.gemms} ({gemm_ms:.3f} ms each)", "errors": errs}
    for k, r in res.items():
        out_rec[k] = {"idle_ms": round(statistics.median(r["idle"]), 4),
                      "contended_ms_median": round(statistics.median(r["lat"]), 4),
                      "contended_ms_min": round(min(r["lat"]), 4),
                      "contended_ms_max": round(max(r["lat"]), 4),
                      "gemm_queue_ms": round(statistics.median(r["gemm"]), 4)}
    print(json.dumps(out_rec), flush=True)


if __name__ == "__main__":
    main()
