"""Row-split GEMMs for odd token counts (the SFT recipe's packed windows, M ~ 4.3 k): hipBLASLt
runs M = 4096 at ~1.3-1.6 PF/s but M = 4300 at ~0.7-1.1 (bench_sft_gemm_pad.py). Times the LLaMA-7B
layer GEMMs (forward X @ W^T and dgrad dY @ W, bf16, torch.mm with out= row slices) issued whole
vs split into row blocks of a multiple of ``q`` plus the remainder. One JSON line per M.

    python benchmarks/bench_sft_gemm_split.py
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


def blocks(M, q):
    if q == 0 or M <= q:
        return [(0, M)]
    head = (M // q) * q
    return [(0, head)] + ([(head, M)] if head < M else [])


def main():
    dev = torch.device("cuda")
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    for M in (4300, 4237, 4608, 5000, 6100, 8600, 3900):
        rec = {"M": M}
        for q in (0, 4096, 2048, 1024):
            tot_f = tot_ms = 0.0
            for k, (n, kk) in shapes.items():
                x = torch.randn(M, kk, device=dev, dtype=torch.bfloat16)
                g = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
                yo = torch.empty(M, n, device=dev, dtype=torch.bfloat16)
                do = torch.empty(M, kk, device=dev, dtype=torch.bfloat16)
                w = ws[k]
                bl = blocks(M, q)

                def fwd():
                    for a, b in bl:
                        torch.mm(x[a:b], w.t(), out=yo[a:b])

                def dgr():
                    for a, b in bl:
                        torch.mm(g[a:b], w, out=do[a:b])
                tot_ms += timeit(fwd) + timeit(dgr)
                tot_f += 4.0 * M * n * kk
            rec[f"q{q}_ms"] = round(tot_ms, 3)
            rec[f"q{q}_tf"] = round(tot_f / tot_ms / 1e9, 1)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
