"""Forward linear GEMM microbenchmark: the hand-written MFMA kernel (csrc/kernels/linear_gemm.hip)
against torch.nn.functional.linear (hipBLASLt, TunableOp table if enabled) on the GPT-2 345M
training shapes at micro-batch 32 (M = 32768 tokens), plus the fused fc1 + bias + GeLU epilogue
against hipBLASLt + the separate bias-GeLU kernel.

    python benchmarks/bench_linear.py [--m 32768]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402
from smdt_amd.ops import functional as SF  # noqa: E402


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(iters):
        ev[0].record()
        fn()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=32768)
    a = p.parse_args()
    C = _ext.ext()
    M = a.m
    torch.manual_seed(0)
    for name, N, K in (("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
                       ("lm_head", 50304, 1024)):
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
        t_ours = timeit(lambda: C.linear_fwd(x, w, b, 1, 8))
        t_ours4 = timeit(lambda: C.linear_fwd(x, w, b, 1, 4))
        t_lib = timeit(lambda: F.linear(x, w, b))
        fl = 2.0 * M * N * K
        rec = {"gemm": name, "M": M, "N": N, "K": K, "ours_ms": t_ours, "ours4_ms": t_ours4, "hipblaslt_ms": t_lib,
               "ours_tflops": fl / t_ours / 1e9, "ours4_tflops": fl / t_ours4 / 1e9, "hipblaslt_tflops": fl / t_lib / 1e9}
        if name == "fc1":
            t_fused = timeit(lambda: C.linear_fwd(x, w, b, 2, 8))
            rec["fused4_bias_gelu_ms"] = timeit(lambda: C.linear_fwd(x, w, b, 2, 4))
            t_unf = timeit(lambda: SF.bias_gelu(F.linear(x, w), b, "tanh"))
            rec.update({"fused_bias_gelu_ms": t_fused, "hipblaslt_plus_bias_gelu_ms": t_unf})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
