"""Weight-gradient GEMM variants on the GPT-2 345M shapes (M = 16384 tokens).

dW[N, K] (+)= dY[M, N]^T X[M, K] — the reduction index M is the slow (row) index of BOTH
operands. Compares: the hipBLASLt beta=1 fp32 accumulate we ship, torch bf16-out NT, and the
"transpose then TN" formulation (+ the transpose cost). Prints one JSON line per shape.
"""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from smdt_amd.ops import _ext  # noqa: E402

SHAPES = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096),
          "lm_head": (50304, 1024), "square_256_tiles": (4096, 4096)}


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
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    M = 16384
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    C = _ext.ext()
    for name, (N, K) in SHAPES.items():
        if only and name not in only:
            continue
        g = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        mg = torch.zeros(N, K, device="cuda", dtype=torch.float32)
        flops = 2.0 * M * N * K
        r = {"shape": name, "M": M, "N": N, "K": K}
        r["blaslt_fp32_acc_us"] = timeit(lambda: C.wgrad_accumulate(mg, g, x))
        r["mfma_fp32_acc_us"] = timeit(lambda: C.wgrad_mfma(mg, g, x, 0))
        r["mfma_nosplit_us"] = timeit(lambda: C.wgrad_mfma(mg, g, x, 1))
        # correctness: one accumulate into zeros vs an fp32 reference on a 2048-row slice
        ms = 2048
        ref = g[:ms].float().t() @ x[:ms].float()
        out = torch.zeros_like(mg)
        C.wgrad_mfma(out, g[:ms].contiguous(), x[:ms].contiguous(), 0)
        r["mfma_max_rel_err"] = float((out - ref).abs().max() / ref.abs().max())
        r["torch_nt_bf16_us"] = timeit(lambda: torch.mm(g.t(), x))
        gt, xt = g.t().contiguous(), x.t().contiguous()
        r["torch_tn_bf16_us"] = timeit(lambda: torch.mm(gt, xt.t()))
        r["transpose_both_us"] = timeit(lambda: (g.t().contiguous(), x.t().contiguous()))
        for k in list(r):
            if k.endswith("_us") and k != "transpose_both_us":
                r[k.replace("_us", "_tflops")] = round(flops / (r[k] * 1e-6) / 1e12, 1)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


def grouped(layers=4):
    """Deferred-wgrad form: every layer's QKV / proj / fc1 / fc2 weight gradient in ONE grouped
    launch (no split-K) vs the same GEMMs one by one (hipBLASLt and the split-K MFMA kernel)."""
    M = 16384
    C = _ext.ext()
    probs = []
    for _ in range(layers):
        for name in ("qkv", "proj", "fc1", "fc2"):
            N, K = SHAPES[name]
            probs.append((torch.zeros(N, K, device="cuda"), torch.randn(M, N, device="cuda", dtype=torch.bfloat16),
                          torch.randn(M, K, device="cuda", dtype=torch.bfloat16)))
    mgs, dys, xs = (list(t) for t in zip(*probs))
    flops = sum(2.0 * M * d.shape[1] * x.shape[1] for d, x in zip(dys, xs))
    r = {"shape": f"grouped_{layers}_layers", "problems": len(probs)}
    r["grouped_us"] = timeit(lambda: C.wgrad_grouped(mgs, dys, xs))
    r["blaslt_each_us"] = timeit(lambda: [C.wgrad_accumulate(m, d, x) for m, d, x in probs])
    r["mfma_each_us"] = timeit(lambda: [C.wgrad_mfma(m, d, x, 0) for m, d, x in probs])
    for k in list(r):
        if k.endswith("_us"):
            r[k.replace("_us", "_tflops")] = round(flops / (r[k] * 1e-6) / 1e12, 1)
    # correctness of the grouped path on a 1024-row slice
    sl = [(torch.zeros_like(m), d[:1024].contiguous(), x[:1024].contiguous()) for m, d, x in probs[:4]]
    C.wgrad_grouped([a for a, _, _ in sl], [b for _, b, _ in sl], [c for _, _, c in sl])
    r["grouped_max_rel_err"] = max(float((a - b.float().t() @ c.float()).abs().max() / (b.float().t() @ c.float()).abs().max())
                                   for a, b, c in sl)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1].startswith("grouped"):
        grouped(int(sys.argv[2]) if len(sys.argv) > 2 else 4)
    else:
        main()
