"""W GEMM fillers (parallel/tensor_parallel.DeferredWgrad.fill_one) against the grouped flush, at
the GPT-2 345M tp2 stage shapes (mbs 32 x seq 1024 = 32,768 tokens per micro-batch; per layer the
weight gradients of qkv [1536, 1024], proj [1024, 512], fc1 [2048, 1024], fc2 [1024, 2048]).

Times, on one GPU, the W work of one micro-batch of a 13-layer stage:
  * ``flush``: ONE grouped launch of all 52 items (the split schedules' per-pass flush);
  * ``fill<cus>``: 52 single-item launches, each with its tail split sized for ``cus`` CUs (the
    filler form; 192 = the CUs a relay transfer leaves);
  * ``fill<cus>_x<k>``: k items per launch;
  * the fillers beside a paced copy holding 64 CUs for the whole run (the relay stand-in).
Prints one JSON line: microseconds and effective PFLOP/s per form.

    python benchmarks/bench_wfill.py [--layers 13] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402

SHAPES = [(1536, 1024), (1024, 512), (2048, 1024), (1024, 2048)]   # (N = out, K = in) per layer


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--layers", type=int, default=13)
    p.add_argument("--tokens", type=int, default=32768)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = a.tokens
    items = []
    for _ in range(a.layers):
        for n, k in SHAPES:
            items.append((torch.zeros(n, k, device=dev, dtype=torch.float32),
                          torch.randn(M, n, device=dev, dtype=torch.bfloat16),
                          torch.randn(M, k, device=dev, dtype=torch.bfloat16)))
    flops = sum(2.0 * M * g.shape[1] * x.shape[1] for _, g, x in items)
    nob = torch.empty(0, device=dev, dtype=torch.float32)

    def flush():
        C.wgrad_grouped([i[0] for i in items], [i[1] for i in items], [i[2] for i in items],
                        [nob] * len(items), [False] * len(items), 0)

    def fill(cus, per=1):
        def run():
            for j in range(0, len(items), per):
                grp = items[j:j + per]
                C.wgrad_grouped([i[0] for i in grp], [i[1] for i in grp], [i[2] for i in grp],
                                [nob] * len(grp), [False] * len(grp), cus)
        return run

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        best = 1e30
        for _ in range(a.reps):
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            best = min(best, s.elapsed_time(e) * 1e3)
        return best

    forms = {"flush": flush, "fill256": fill(256), "fill192": fill(192), "fill192_x2": fill(192, 2),
             "fill192_x4": fill(192, 4)}
    res = {}
    for name, fn in forms.items():
        us = timed(fn)
        res[name] = {"us": round(us, 1), "pflops": round(flops / us / 1e9, 3)}
        print(f"{name:14s} {us:9.1f} us  {flops / us / 1e9:.3f} PF/s", flush=True)
    # beside a paced copy holding 64 CUs (the relay stand-in) for the whole measurement
    side = torch.cuda.Stream(dev)
    buf = torch.empty(64 << 20, device=dev, dtype=torch.uint8)
    out = torch.empty_like(buf)
    for name in ("fill192", "fill192_x2"):
        fn = forms[name]
        us0 = res["flush"]["us"]
        fn_start, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            C.paced_copy(out, buf, 64, int(us0 * 3000))      # holds 64 CUs ~3x the flush time
        fn_start.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        us = fn_start.elapsed_time(e) * 1e3
        res[name + "_beside_64cu_copy"] = {"us": round(us, 1), "pflops": round(flops / us / 1e9, 3)}
        print(f"{name + '_beside':14s} {us:9.1f} us  {flops / us / 1e9:.3f} PF/s", flush=True)
    print(json.dumps({"tokens": M, "layers": a.layers, "items": len(items), "gflop": round(flops / 1e9, 1), **res}))


if __name__ == "__main__":
    main()
