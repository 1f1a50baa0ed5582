"""Dgrad GEMM layout: dX = dY W (W [out, in] row-major, hipBLASLt "NN") against
dX = F.linear(dY, Wt) with Wt = W^T made contiguous right before the GEMM ("TN" + a transpose
copy), at the GPT-2 345M shapes (M = 65536 tokens, micro-batch 64), TunableOp table loaded as in
bench.py. Prints one JSON line per shape; the TN total includes the transpose (our LDS
tile kernel, transpose.hip; torch's strided copy is timed beside it)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65536)
    ap.add_argument("--no-tunable", action="store_true")
    a = ap.parse_args()
    if not a.no_tunable:
        import torch.cuda.tunable as tun
        tun.enable(True)
        tun.tuning_enable(False)
        tun.read_file(os.path.join(ROOT, "profiles", "tunableop", "gfx950_gpt345m_results.csv"))
    M = a.m
    sys.path.insert(0, ROOT)
    from smdt_amd.ops import _ext
    C = _ext.ext() if _ext.available() else None
    tot_nn = tot_tn = 0.0
    # (name, out, in): dX [M, in] = dY [M, out] @ W [out, in]
    for name, O, I in (("qkv", 3072, 1024), ("proj", 1024, 1024), ("fc1", 4096, 1024), ("fc2", 1024, 4096),
                       ("lm_head", 50304, 1024)):
        g = torch.randn(M, O, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(O, I, device="cuda", dtype=torch.bfloat16) * 0.02
        ref = g.matmul(w)
        alt = F.linear(g, w.t().contiguous())
        err = (ref.float() - alt.float()).abs().max().item()
        t_nn = timeit(lambda: g.matmul(w))
        t_tr_torch = timeit(lambda: w.t().contiguous())
        t_tr = timeit(lambda: C.transpose2d(w)) if C is not None else t_tr_torch
        assert C is None or torch.equal(C.transpose2d(w), w.t().contiguous())
        wt = w.t().contiguous()
        t_tn = timeit(lambda: F.linear(g, wt))
        fl = 2.0 * M * O * I
        n = 1 if name == "lm_head" else 24
        tot_nn += n * t_nn
        tot_tn += n * (t_tn + t_tr)
        print(json.dumps({"gemm": name, "nn_ms": round(t_nn, 4), "tn_ms": round(t_tn, 4), "transpose_ms": round(t_tr, 4), "torch_transpose_ms": round(t_tr_torch, 4),
                          "nn_tflops": round(fl / t_nn / 1e9, 1), "tn_tflops": round(fl / t_tn / 1e9, 1),
                          "max_abs_diff": err}), flush=True)
    print(json.dumps({"per_step_ms_nn": round(tot_nn, 3), "per_step_ms_tn_incl_transpose": round(tot_tn, 3)}), flush=True)


if __name__ == "__main__":
    main()
