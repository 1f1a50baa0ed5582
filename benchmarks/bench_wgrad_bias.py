"""Grouped weight-gradient launch with and without the fused bias column sums.

One launch of the bench's deferred-wgrad group shape: ``--layers`` GPT-2 345M layers (QKV 3072 x
1024, proj 1024 x 1024, fc1 4096 x 1024, fc2 1024 x 4096 main_grads; M = 65,536 tokens), timed
(a) without bias targets, (b) with the QKV / fc1 bias targets the training step passes, (c) with
bias targets on every problem. Prints one JSON line; the bias sums are checked against fp32
column sums of dY.

    python benchmarks/bench_wgrad_bias.py [--layers 5] [--m 65536]
"""
import argparse
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=5)
    ap.add_argument("--m", type=int, default=65536)
    a = ap.parse_args()
    C = _ext.ext()
    dev = torch.device("cuda")
    M = a.m
    shapes = [("qkv", 3072, 1024, True), ("proj", 1024, 1024, False), ("fc1", 4096, 1024, True),
              ("fc2", 1024, 4096, False)]
    mgs, dys, xs, bias_some, bias_all = [], [], [], [], []
    empty = torch.empty(0, device=dev, dtype=torch.float32)
    xin = {k: torch.randn(M, k, device=dev, dtype=torch.bfloat16) for k in (1024, 4096)}
    for _ in range(a.layers):
        for name, n, k, has_bias in shapes:
            mgs.append(torch.zeros(n, k, device=dev))
            dys.append(torch.randn(M, n, device=dev, dtype=torch.bfloat16))
            xs.append(xin[k])
            b = torch.zeros(n, device=dev)
            bias_all.append(b)
            bias_some.append(b if has_bias else empty)
    tiles = sum(-(-m.shape[0] // 256) * -(-m.shape[1] // 256) for m in mgs)
    flops = sum(2.0 * M * m.shape[0] * m.shape[1] for m in mgs)
    res = {"layers": a.layers, "M": M, "tiles": tiles}
    for label, biases in (("no_bias", []), ("bias_qkv_fc1", bias_some), ("bias_all", bias_all)):
        ms = timeit(lambda: C.wgrad_grouped(mgs, dys, xs, biases))
        res[f"{label}_ms"] = round(ms, 3)
        res[f"{label}_tflops"] = round(flops / (ms * 1e-3) / 1e12, 1)
    # correctness of the fused sums: one launch into zeroed targets vs fp32 column sums
    for b in bias_all:
        b.zero_()
    C.wgrad_grouped(mgs, dys, xs, bias_all)
    err = max(float((b - d.float().sum(0)).abs().max() / d.float().sum(0).abs().max().clamp(min=1e-6))
              for b, d in zip(bias_all, dys))
    res["bias_max_rel_err"] = err
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
