"""Weight-gradient GEMM variants on the GPT-2 345M shapes (M = 16384 tokens).

dW[N, K] (+)= dY[M, N]^T X[M, K] — the reduction index M is the slow (row) index of BOTH
operands. Compares: the hipBLASLt beta=1 fp32 accumulate we ship, torch bf16-out NT, and the
"transpose then TN" formulation (+ the transpose cost). Prints one JSON line per shape.
"""
import json
import sys

import torch

sys.path.insert(0, ".")
from smdt_amd.ops import _ext  # noqa: E402

SHAPES = {"qkv": (3072, 1024), "proj": (1024, 1024), "fc1": (4096, 1024), "fc2": (1024, 4096),
          "lm_head": (50304, 1024)}


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
    C = _ext.ext()
    for name, (N, K) in SHAPES.items():
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


if __name__ == "__main__":
    main()
