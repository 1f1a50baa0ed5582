#!/usr/bin/env python3
"""LLaMA-7B linear GEMMs on one MI355X: hipBLASLt heuristics vs TunableOp-tuned, at the token
counts an Alpaca SFT micro-batch produces (M = micro-batch x padded length).

Forward y = x W^T ([M, K] x [N, K]^T) and TN dgrad dX = dY W ([M, N] x [N, K]) for the QKV / O /
gate+up / down / LM-head shapes. Prints one JSON line per (shape, M) with TF/s of both.
``--tune`` turns TunableOp on (writes the table to --out); without it the library heuristics run.
"""
import argparse
import json
import os

import torch

SHAPES = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008),
          "lm_head": (32000, 4096)}


def timeit(fn, iters=10):
    for _ in range(3):
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
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--out", default="gpurun_out/llama_tunableop.csv")
    ap.add_argument("--m", default="4096,8192,16384")
    a = ap.parse_args()
    if a.tune:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(30)
        tun.set_filename(os.path.abspath(a.out))
    for M in [int(v) for v in a.m.split(",")]:
        for name, (N, K) in SHAPES.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
            wt = w.t().contiguous()
            f_ms = timeit(lambda: torch.nn.functional.linear(x, w))
            d_ms = timeit(lambda: torch.nn.functional.linear(dy, wt))
            fl = 2.0 * M * N * K
            print(json.dumps({"M": M, "shape": name, "N": N, "K": K, "tuned": a.tune,
                              "fwd_tflops": round(fl / f_ms / 1e9, 1), "dgrad_tn_tflops": round(fl / d_ms / 1e9, 1)}),
                  flush=True)
    if a.tune:
        import torch.cuda.tunable as tun
        tun.write_file()


if __name__ == "__main__":
    main()
