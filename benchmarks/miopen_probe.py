#!/usr/bin/env python3
"""Which MIOpen convolution solutions run for the Oxford-Pet ResNet-50 convolutions (bf16,
channels-last), and how fast: one 3x3 and one 1x1 convolution of the ResNet-50 stage-1 shape,
forward + backward timed after a warm-up, under the same ``cudnn.benchmark = True`` the vision
bench uses. Run it with ``MIOPEN_LOG_LEVEL=4`` (warnings) / ``MIOPEN_ENABLE_LOGGING=1`` to see
MIOpen's find results and any solver that fails to build.

    python benchmarks/miopen_probe.py [--nchw] [--fp32] [--no-benchmark]
"""
import argparse
import json
import time

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nchw", action="store_true")
    ap.add_argument("--fp32", action="store_true")
    ap.add_argument("--no-benchmark", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = not a.no_benchmark
    dt = torch.float32 if a.fp32 else torch.bfloat16
    mf = torch.contiguous_format if a.nchw else torch.channels_last
    dev = torch.device("cuda")
    out = {"dtype": str(dt), "layout": "nchw" if a.nchw else "nhwc", "benchmark": not a.no_benchmark}
    for name, (cin, cout, k) in {"3x3": (64, 64, 3), "1x1": (256, 64, 1)}.items():
        x = torch.randn(64, cin, 56, 56, device=dev, dtype=dt).to(memory_format=mf).requires_grad_()
        w = torch.randn(cout, cin, k, k, device=dev, dtype=dt).to(memory_format=mf).requires_grad_()

        def step():
            y = F.conv2d(x, w, padding=k // 2)
            y.backward(torch.ones_like(y))
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        first = time.perf_counter() - t0
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.iters * 1e3
        flops = 3 * 2 * 64 * 56 * 56 * cin * cout * k * k
        out[name] = {"first_call_s": round(first, 2), "ms_fwd_bwd": round(ms, 3), "tflops": round(flops / ms / 1e9, 1)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
