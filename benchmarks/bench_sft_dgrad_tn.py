"""SFT dgrad form at the LLaMA-7B layer shapes and packed-window token counts: dY @ W as an NN
GEMM vs the TN form F.linear(dY, W^T) the framework uses (tensor_parallel.dgrad) plus the W^T
transpose, which the fused accumulation window pays once per weight per step. One JSON line
per M.

    python benchmarks/bench_sft_dgrad_tn.py
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from smdt_amd.ops import _ext  # noqa: E402
from smdt_amd.parallel import tensor_parallel as tp  # noqa: E402


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
    C = _ext.ext()
    dev = torch.device("cuda")
    if "--gpt2" in sys.argv:   # GPT-2 345M at the bench (M = 65536) and tp2 ring-chunk (16384) shapes
        for M, tpn in ((65536, 1), (16384, 2)):
            rec = {"M": M, "tp": tpn}
            for k, (n, kk) in {"qkv": (3072 // tpn, 1024), "proj": (1024, 1024 // tpn), "fc1": (4096 // tpn, 1024),
                               "fc2": (1024, 4096 // tpn)}.items():
                w = torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02
                wt = C.transpose2d(w)
                g = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
                rec[k] = {"nn_ms": round(timeit(lambda: torch.mm(g, w)), 4),
                          "tn_ms": round(timeit(lambda: tp.linear_rows(g, wt)), 4),
                          "transpose_ms": round(timeit(lambda: C.transpose2d(w)), 4)}
            print(json.dumps(rec), flush=True)
        return
    shapes = {"qkv": (12288, 4096), "o": (4096, 4096), "gate_up": (22016, 4096), "down": (4096, 11008)}
    ws = {k: torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    wts = {k: C.transpose2d(w) for k, w in ws.items()}
    t_tr = sum(timeit(lambda: C.transpose2d(w)) for w in ws.values())
    for M in (3900, 4096, 4300, 4608, 8600):
        rec = {"M": M, "transpose_ms": round(t_tr, 3)}
        nn = tn = 0.0
        for k, (n, kk) in shapes.items():
            g = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
            w, wt = ws[k], wts[k]
            a = timeit(lambda: torch.mm(g, w))
            b = timeit(lambda: tp.linear_rows(g, wt))
            rec[k] = {"nn_ms": round(a, 4), "tn_ms": round(b, 4)}
            nn += a
            tn += b
        rec["nn_ms"], rec["tn_ms"], rec["tn_plus_transpose_ms"] = round(nn, 3), round(tn, 3), round(tn + t_tr, 3)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
