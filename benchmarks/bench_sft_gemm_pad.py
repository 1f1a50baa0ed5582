"""hipBLASLt rate of the LLaMA-7B layer GEMMs at the SFT recipe's token counts (padding-free
packing: M = real tokens of a fused window, ~4.3 k at NB4's 4 x GA 8), and with M rounded up to a
multiple of 256 / 512. Forward X[M, K] @ W[N, K]^T and dgrad dY[M, N] @ W[N, K], bf16, torch.mm
(the recipe's path). Prints one JSON line of TF/s per (M, GEMM).

    python benchmarks/bench_sft_gemm_pad.py
"""
import json

import torch


def timeit(fn, iters=20):
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
    dev = torch.device("cuda")
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    res = {}
    for M in (4300, 4352, 4608, 4237, 4096, 8600, 8704):
        row = {}
        tot_f = tot_ms = 0.0
        for k, (n, kk) in shapes.items():
            x = torch.randn(M, kk, device=dev, dtype=torch.bfloat16)
            g = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
            w = ws[k]
            f = 2.0 * M * n * kk
            ms_f = timeit(lambda: torch.mm(x, w.t()))
            ms_d = timeit(lambda: torch.mm(g, w))
            row[k] = {"fwd_tf": round(f / ms_f / 1e9, 1), "dgrad_tf": round(f / ms_d / 1e9, 1)}
            tot_f += 2 * f
            tot_ms += ms_f + ms_d
        row["all_tf"] = round(tot_f / tot_ms / 1e9, 1)
        row["all_ms"] = round(tot_ms, 3)
        res[str(M)] = row
        print(json.dumps({"M": M, **row}), flush=True)


if __name__ == "__main__":
    main()
