"""HBM rate of the step's elementwise kernels at the GPT-2 345M bench shapes (one GPU), plus the
SFT recipe's SwiGLU and the LM-head cross-entropy. (A 4-vectors-in-flight CE backward measured
no faster, 2.51 vs 2.47 ms at [65536, 50304], and was not kept: profiles/r4_swiglu_2d/ce_unroll.log,
in git history.)

bias-GeLU forward / backward on [65536, 4096] bf16 (fc1 output; backward without d(bias): the
grouped wgrad makes it), the fused bias-dropout-residual LayerNorm forward and its backward on
[65536, 1024]. Prints one JSON line with ms and TB/s per kernel (bytes = what the kernel must read
+ write). (bias_act.hip documents the launch shape).

    python benchmarks/bench_elementwise.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, ".")
from smdt_amd.ops import _ext  # noqa: E402
from smdt_amd.ops import functional as SF  # noqa: E402


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
    res = {}
    T, F, H = 65536, 4096, 1024
    x = torch.randn(T, F, device=dev, dtype=torch.bfloat16)
    b = torch.randn(F, device=dev, dtype=torch.bfloat16)
    dy = torch.randn_like(x)
    nb = x.numel() * 2
    ms = timeit(lambda: C.bias_act_fwd(x, b, 0))
    res["bias_gelu_fwd"] = {"ms": round(ms, 4), "TBps": round(2 * nb / ms / 1e9, 2)}
    ms = timeit(lambda: C.bias_act_bwd(dy, x, b, 0, False, None))
    res["bias_gelu_bwd"] = {"ms": round(ms, 4), "TBps": round(3 * nb / ms / 1e9, 2)}
    # correctness of the selected form vs fp32
    y = C.bias_act_fwd(x[:1024], b, 0).float()
    z = x[:1024].float() + b.float()
    ref = 0.5 * z * (1 + torch.tanh(0.7978845608028654 * (z + 0.044715 * z ** 3)))
    res["bias_gelu_fwd_max_err"] = float((y - ref).abs().max())
    del x, dy
    # LayerNorm (bias + dropout + residual fused) forward / backward
    a = torch.randn(T, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(T, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    bb = torch.zeros(H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    hb = torch.zeros(H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    nh = a.numel() * 2
    try:
        fwd = lambda: SF.bias_dropout_add_norm(a, hb, r, w, bb, 0.1, True)  # noqa: E731
        y, s_ = fwd()
        ms = timeit(fwd)
        # x, residual read; s and y written
        res["ln_fwd"] = {"ms": round(ms, 4), "TBps": round(4 * nh / ms / 1e9, 2)}
        g1, g2 = torch.randn_like(y), torch.randn_like(s_)
        ms = timeit(lambda: torch.autograd.grad((y, s_), (a, r), (g1, g2), retain_graph=True))
        res["ln_bwd_incl_autograd"] = {"ms": round(ms, 4)}
    except Exception as e:  # noqa: BLE001
        res["ln_error"] = repr(e)[:200]
    # SwiGLU at the LLaMA-7B SFT shape (packed window ~4.3 k tokens, ffn 11008)
    xs = torch.randn(4300, 2 * 11008, device=dev, dtype=torch.bfloat16)
    ds = torch.randn(4300, 11008, device=dev, dtype=torch.bfloat16)
    ns = ds.numel() * 2
    ms = timeit(lambda: C.swiglu_fwd(xs))
    res["swiglu_fwd"] = {"ms": round(ms, 4), "TBps": round(3 * ns / ms / 1e9, 2)}
    ms = timeit(lambda: C.swiglu_bwd(ds, xs))
    res["swiglu_bwd"] = {"ms": round(ms, 4), "TBps": round(5 * ns / ms / 1e9, 2)}
    del xs, ds
    # vocab-parallel CE backward at the bench's LM head: [65536, 50304] bf16 logits -> dlogits
    lg = torch.randn(T, 50304, device=dev, dtype=torch.bfloat16)
    tg = torch.randint(0, 50257, (T,), device=dev)
    mx, se, _ = C.ce_stats(lg, tg, 0, 50257)
    dl = torch.ones(T, device=dev)
    out = torch.empty_like(lg)
    nl = lg.numel() * 2
    ms = timeit(lambda: C.ce_bwd(lg, tg, mx, se, dl, out, 0, -100, 50257))
    res["ce_bwd"] = {"ms": round(ms, 4), "TBps": round(2 * nl / ms / 1e9, 2)}
    ms = timeit(lambda: C.ce_stats(lg, tg, 0, 50257))
    res["ce_stats"] = {"ms": round(ms, 4), "TBps": round(nl / ms / 1e9, 2)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
