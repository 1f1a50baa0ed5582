"""Flash-attention microbenchmark: smdt_amd HIP kernels vs torch SDPA on the same random data.

python benchmarks/bench_attention.py [--b 16 --h 16 --s 1024 --d 64 --causal 1]
Reports fwd / bwd times and TFLOP/s (causal FLOPs counted as half of the dense 4*B*H*S^2*D).
"""
import argparse
import json
import math
import time

import torch
import torch.nn.functional as F

import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if "--ext" in sys.argv:
    # A/B builds: load an alternate kernel library (e.g. benchmarks/bin/ab_ref_C.so, the same
    # sources before a change) as smdt_amd._C before anything imports the in-tree one
    import importlib.util
    _p = sys.argv[sys.argv.index("--ext") + 1]
    _spec = importlib.util.spec_from_file_location("smdt_amd._C", _p)
    _m = importlib.util.module_from_spec(_spec)
    import smdt_amd  # noqa: E402,F401
    sys.modules["smdt_amd._C"] = _m
    _spec.loader.exec_module(_m)
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
    p.add_argument("--b", type=int, default=16)
    p.add_argument("--h", type=int, default=16)
    p.add_argument("--hkv", type=int, default=0)
    p.add_argument("--s", type=int, default=1024)
    p.add_argument("--d", type=int, default=64)
    p.add_argument("--causal", type=int, default=1)
    p.add_argument("--sdpa", type=int, default=1)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--ext", default=None, help="alternate _C.so for A/B runs")
    a = p.parse_args()
    B, H, S, D = a.b, a.h, a.s, a.d
    Hkv = a.hkv or H
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    flops = 4 * B * H * S * S * D * (0.5 if a.causal else 1.0)
    res = {"shape": [B, S, H, Hkv, D], "causal": bool(a.causal), "dropout": a.dropout}

    def ours_f():
        return SF.flash_attention(q, k, v, 1 / math.sqrt(D), bool(a.causal), dropout_p=a.dropout)
    o = ours_f()
    tf = timeit(lambda: ours_f())
    tb = timeit(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True))
    res["ours_fwd_ms"], res["ours_bwd_ms"] = tf, tb
    res["ours_fwd_tflops"], res["ours_bwd_tflops"] = flops / tf / 1e9, 2.5 * flops / tb / 1e9
    if a.sdpa and Hkv == H and a.dropout == 0:
        qt, kt, vt = (t.detach().transpose(1, 2).contiguous().requires_grad_() for t in (q, k, v))
        dot = do.transpose(1, 2).contiguous()
        try:
            os2 = F.scaled_dot_product_attention(qt, kt, vt, is_causal=bool(a.causal))
            sf = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=bool(a.causal)))
            sb = timeit(lambda: torch.autograd.grad(os2, (qt, kt, vt), dot, retain_graph=True))
            res["sdpa_fwd_ms"], res["sdpa_bwd_ms"] = sf, sb
            res["sdpa_fwd_tflops"], res["sdpa_bwd_tflops"] = flops / sf / 1e9, 2.5 * flops / sb / 1e9
            res["max_abs_diff_vs_sdpa"] = (os2.transpose(1, 2) - o).abs().max().item()
        except Exception as e:  # pragma: no cover
            res["sdpa_error"] = repr(e)[:200]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
